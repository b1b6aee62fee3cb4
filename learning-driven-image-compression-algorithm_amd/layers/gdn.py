"""compressai-style GDN (reference layers/gdn.py:26-75), the normalisation used
inside ResidualBlockWithStride: out = x * rsqrt(beta' + gamma' x^2)
(inverse: x * sqrt(...)).  Runs as lic_gdn_prepare + one lic_conv2d_fwd launch
(1x1 GEMM over x^2 with the rsqrt/sqrt * x epilogue, optional fused residual).
"""
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
from .._ffi import EPI_GDN_RSQRT, EPI_GDN_SQRT
from ..functional import Act
from ..ops import NonNegativeParametrizer

__all__ = ["GDN"]


class GDN(nn.Module):
    def __init__(self, in_channels: int, inverse: bool = False, beta_min: float = 1e-6, gamma_init: float = 0.1):
        super().__init__()
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        beta = self.beta_reparam.init(torch.ones(in_channels))
        self.beta = nn.Parameter(beta)
        self.gamma_reparam = NonNegativeParametrizer()
        gamma = self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels))
        self.gamma = nn.Parameter(gamma)

        self._refresh_consts()

    def _refresh_consts(self):
        # host copies of the (constant) bound / pedestal buffers: no device sync per call
        self._consts = (float(self.beta_reparam.lower_bound.bound.cpu().item()),
                        float(self.gamma_reparam.lower_bound.bound.cpu().item()),
                        float(self.beta_reparam.pedestal.cpu().item()))

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self._refresh_consts()

    def packed(self, dtype) -> Fn.ConvPack:
        # ops/parametrizers.py:48-51 evaluated on device (lic_gdn_prepare), cached per parameter version.
        key = (dtype, self.beta.data_ptr(), self.beta._version, self.gamma.data_ptr(), self.gamma._version)
        cache = self.__dict__.setdefault("_lic_packs", {})
        if key not in cache:
            cache.clear()
            bb, gb, ped = self._consts
            cache[key] = Fn.gdn_prepare(self.beta, self.gamma, bb, gb, ped, dtype)
        return cache[key]

    def run(self, x: Act, out: Optional[Act] = None, r1: Optional[Act] = None) -> Act:
        pk = self.packed(x.dtype)
        return Fn.gdn(x, pk, EPI_GDN_SQRT if self.inverse else EPI_GDN_RSQRT, out, r1)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()
