"""GDN / IGDN of reference model/gdn.py:29-156: GDN out = x / sqrt(n),
IGDN out = x * sqrt(n), n = beta' + conv1x1(x^2, gamma'), with
beta' = max(beta, sqrt(1e-6 + offset^2))^2 - offset^2, gamma' = max(gamma, offset)^2 - offset^2.

The reference's LowerBound materialises ``torch.ones(size) * bound`` on the host
and copies it to the device on every call (model/gdn.py:14-15); here the bound
is a scalar argument of the on-device lic_gdn_prepare kernel.
"""
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
from .._ffi import EPI_GDN_DIV, EPI_GDN_SQRT
from ..functional import Act

__all__ = ["GDN", "IGDN"]


class _GDNBase(nn.Module):
    _inverse_math = False

    def __init__(self, ch, inverse=False, beta_min=1e-6, gamma_init=.1, reparam_offset=2 ** -18):
        super().__init__()
        self.inverse = inverse
        self.beta_min = beta_min
        self.gamma_init = gamma_init
        self.register_buffer("reparam_offset", torch.FloatTensor([reparam_offset]))
        self.register_buffer("pedestal", self.reparam_offset ** 2)
        # model/gdn.py:52-53: evaluated in fp32 tensor arithmetic at build time
        self._refresh_consts()
        self.beta = nn.Parameter(torch.sqrt(torch.ones(ch) + self.pedestal))
        self.gamma = nn.Parameter(torch.sqrt(self.gamma_init * torch.eye(ch) + self.pedestal))

    def _refresh_consts(self):
        ro = self.reparam_offset.detach().cpu()
        # beta_bound / gamma_bound are fixed at build() from the initial offset (model/gdn.py:52-54)
        if not hasattr(self, "_beta_bound"):
            self._beta_bound = float(((self.beta_min + ro ** 2) ** .5).item())
            self._gamma_bound = float(ro.item())
        self._pedestal = float(self.pedestal.detach().cpu().item())

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self._refresh_consts()

    def packed(self, dtype) -> Fn.ConvPack:
        key = (dtype, self.beta.data_ptr(), self.beta._version, self.gamma.data_ptr(), self.gamma._version)
        cache = self.__dict__.setdefault("_lic_packs", {})
        if key not in cache:
            cache.clear()
            cache[key] = Fn.gdn_prepare(self.beta, self.gamma, self._beta_bound, self._gamma_bound,
                                        self._pedestal, dtype)
        return cache[key]

    def run(self, x: Act, out: Optional[Act] = None, r1: Optional[Act] = None) -> Act:
        mode = EPI_GDN_SQRT if self._inverse_math else EPI_GDN_DIV
        return Fn.gdn(x, self.packed(x.dtype), mode, out, r1)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()


class GDN(_GDNBase):
    """y = x / sqrt(beta + sum_j gamma[i, j] x_j^2) (model/gdn.py:29-92)."""
    _inverse_math = False


class IGDN(_GDNBase):
    """y = x * sqrt(beta + sum_j gamma[i, j] x_j^2) (model/gdn.py:94-156)."""
    _inverse_math = True
