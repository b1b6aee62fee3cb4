"""Restatements of the compressai layers the reference imports but does not
vendor (compressai 1.2.x: compressai/layers/layers.py, compressai/entropy_models),
with compressai's parameter names, executed on liblic.

Call sites: layers/layers.py:14-21,87-102; model/net_ga.py:52-59,153,271,295,746,857.
"""
import os
from typing import Optional

import torch
import torch.nn as nn

from .._ffi import ACT_LRELU, ACT_RELU, EPI_GATE, EPI_RES_ACT
from .. import functional as Fn
from ..functional import Act
from ._conv import Conv2d
from .gdn import GDN
from ..ops import LowerBound

__all__ = ["conv3x3", "conv1x1", "subpel_conv3x3", "ResidualBlock", "ResidualBlockWithStride", "AttentionBlock",
           "EntropyBottleneck", "GaussianConditional"]


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def subpel_conv3x3(in_ch: int, out_ch: int, r: int = 1) -> nn.Sequential:
    """conv3x3(out*r^2) + PixelShuffle(r); the shuffle is fused into the conv's store addressing."""
    return nn.Sequential(Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), nn.PixelShuffle(r))


class ResidualBlock(nn.Module):
    """conv3x3 -> LReLU -> conv3x3 -> LReLU -> + identity (skip 1x1 if in != out)."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None

    def run(self, x: Act, out: Optional[Act] = None, gate_a: Optional[Act] = None,
            gate_r: Optional[Act] = None) -> Act:
        """If gate_a is given the Win_noShift_Attention gate is fused:
        out = gate_a * sigmoid(block(x)) + gate_r."""
        t = self.conv1.run(x, act=ACT_LRELU)
        identity = self.skip.run(x) if self.skip is not None else x
        if gate_a is not None:
            return self.conv2.run(t, out, act=ACT_LRELU, r1=identity, epi=EPI_GATE, g=gate_a, r2=gate_r)
        return self.conv2.run(t, out, act=ACT_LRELU, r1=identity)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()


class ResidualBlockWithStride(nn.Module):
    """conv3x3 s2 -> LReLU -> conv3x3 -> GDN -> + conv1x1 s2 skip (GDN + add fused)."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 2):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch, stride=stride)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv3x3(out_ch, out_ch)
        self.gdn = GDN(out_ch)
        self.skip = conv1x1(in_ch, out_ch, stride=stride) if (stride != 1 or in_ch != out_ch) else None

    def run(self, x: Act, out: Optional[Act] = None, fork: bool = False) -> Act:
        """fork=True (called on the capture stream) and LIC_FORK_SKIP=1: the 1x1 s2 skip on a side stream
        forked from the current one (a sibling of every other fork, never nested), beside conv1 -> conv2;
        joined before the GDN epilogue that adds it.  Same launches, same arithmetic; opt-in because it
        measured neutral (fp32x6 1075.6 / 1074.3 -> 1073.9 / 1076.6 images/s, profiles/r06/fork_skip_ab.txt)."""
        side = None
        if fork and self.skip is not None and Fn.fork_enabled() and os.environ.get("LIC_FORK_SKIP", "0") == "1":
            main = torch.cuda.current_stream(x.t.device)
            side = Fn.aux_stream(x.t.device, "skip")
            side.wait_stream(main)
            with torch.cuda.stream(side):
                identity = self.skip.run(x)
        t = self.conv1.run(x, act=ACT_LRELU)
        t = self.conv2.run(t)
        if side is not None:
            main.wait_stream(side)
            identity.t.record_stream(main)   # allocated on the side stream, read by the GDN launch here
        else:
            identity = self.skip.run(x) if self.skip is not None else x
        return self.gdn.run(t, out, r1=identity)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()


_FUSED_RU = os.environ.get("LIC_FUSED_RU", "1") != "0"   # A/B switch for the fused fp32x6 unit


class _ResidualUnit(nn.Module):
    def __init__(self, N):
        super().__init__()
        self.conv = nn.Sequential(conv1x1(N, N // 2), nn.ReLU(inplace=True), conv3x3(N // 2, N // 2),
                                  nn.ReLU(inplace=True), conv1x1(N // 2, N))
        self.relu = nn.ReLU(inplace=True)

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        if x.dtype == torch.float32 and Fn.split_mode() == 2 and _FUSED_RU:
            # fp32x6: the whole unit in one launch, intermediates in LDS (csrc/resunit_split.hip)
            packs = [self.conv[i].packed(x.dtype) for i in (0, 2, 4)]
            if Fn.resunit_fusable(x, *packs, out=out):
                return Fn.resunit(x, *packs, out=out)
        t = self.conv[0].run(x, act=ACT_RELU)
        t = self.conv[2].run(t, act=ACT_RELU)
        # out = relu(conv(t) + identity): residual added before the activation
        return self.conv[4].run(t, out, r1=x, act=ACT_RELU, epi=EPI_RES_ACT)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()


class AttentionBlock(nn.Module):
    """compressai AttentionBlock(N): x + conv_a(x) * sigmoid(conv_b(x))."""

    def __init__(self, N: int):
        super().__init__()
        self.conv_a = nn.Sequential(_ResidualUnit(N), _ResidualUnit(N), _ResidualUnit(N))
        self.conv_b = nn.Sequential(_ResidualUnit(N), _ResidualUnit(N), _ResidualUnit(N), conv1x1(N, N))


class EntropyBottleneck(nn.Module):
    """Only ``_get_medians()`` influences the reference outputs (net_ga.py:996-1003):
    its likelihoods are computed and discarded.  The parameter / buffer names of
    compressai 1.2 are kept for state_dict compatibility; the factorized-prior MLP
    is not evaluated."""

    def __init__(self, channels: int, init_scale: float = 10, filters=(3, 3, 3, 3), likelihood_bound: float = 1e-9):
        super().__init__()
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())
        self.likelihood_lower_bound = LowerBound(likelihood_bound)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        import math
        for i in range(len(self.filters) + 1):
            init = math.log(math.expm1(1 / scale / filters[i + 1]))
            matrix = torch.Tensor(channels, filters[i + 1], filters[i])
            matrix.data.fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(matrix))
            bias = torch.Tensor(channels, filters[i + 1], 1)
            nn.init.uniform_(bias, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(bias))
            if i < len(self.filters):
                factor = torch.Tensor(channels, filters[i + 1], 1)
                nn.init.zeros_(factor)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(factor))
        self.quantiles = nn.Parameter(torch.Tensor(channels, 1, 3))
        init = torch.Tensor([-self.init_scale, 0, self.init_scale])
        self.quantiles.data = init.repeat(self.quantiles.size(0), 1, 1)
        target = math.log(2 / 1e-9 - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self) -> torch.Tensor:
        return self.quantiles[:, :, 1:2]

    def medians_flat(self) -> torch.Tensor:
        return self.quantiles[:, 0, 1].detach().float().contiguous()


class GaussianConditional(nn.Module):
    """compressai GaussianConditional(None) — buffers kept for state_dict parity; the
    quantise + likelihood math runs in lic_gauss_rate_fwd."""

    def __init__(self, scale_table=None, scale_bound: float = 0.11, tail_mass: float = 1e-9,
                 likelihood_bound: float = 1e-9):
        super().__init__()
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())
        self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.tail_mass = float(tail_mass)
        self.register_buffer("scale_table", torch.Tensor(tuple(float(s) for s in scale_table))
                             if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]) if scale_bound is not None else None)
        self.lower_bound_scale = LowerBound(scale_bound)
        self._scale_bound = float(torch.Tensor([float(scale_bound)]).item())
        self._likelihood_bound = float(torch.Tensor([float(likelihood_bound)]).item())
