"""Conv helpers and Win_noShift_Attention (reference layers/layers.py:36-111)."""
import os
from typing import Optional

import torch
import torch.nn as nn

from ..functional import Act
from ._conv import Conv2d
from .compressai import ResidualBlock
from .win_attention import WinBasedAttention

__all__ = ["conv3x3", "conv7x7", "subpel_conv3x3", "conv1x1", "Win_noShift_Attention"]


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv7x7(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    return Conv2d(in_ch, out_ch, kernel_size=7, stride=stride, padding=3)


def subpel_conv3x3(in_ch: int, out_ch: int, r: int = 1) -> nn.Sequential:
    return nn.Sequential(Conv2d(in_ch, out_ch * r ** 2, kernel_size=3, padding=1), nn.PixelShuffle(r))


def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


class Win_noShift_Attention(nn.Module):
    """out = x + conv_a(x) * sigmoid(conv_b(x)) (layers/layers.py:105-111).
    conv_a = 3 x ResidualBlock; conv_b = WBA, 1x1, WBA, RB, 3x3, WBA, RB, 7x7, WBA, RB.
    The gate and the outer residual are fused into the epilogue of the last conv
    of conv_b; every WBA's shortcut add is fused into its proj launch."""

    def __init__(self, dim, num_heads=8, window_size=8, shift_size=0):
        super().__init__()
        N = dim
        self.conv_a = nn.Sequential(ResidualBlock(N, N), ResidualBlock(N, N), ResidualBlock(N, N))
        wba = lambda: WinBasedAttention(dim=dim, num_heads=num_heads, window_size=window_size, shift_size=shift_size)
        self.conv_b = nn.Sequential(
            wba(), conv1x1(N, N), wba(), ResidualBlock(N, N), conv3x3(N, N), wba(), ResidualBlock(N, N),
            conv7x7(N, N), wba(), ResidualBlock(N, N))

    # maps up to this many pixels (batch x H x W) run conv_a concurrently with conv_b: there every
    # launch is latency-bound (the 16x16 latents); on the big maps both chains fill the GPU alone
    CONCURRENT_MAX_PIX = 16384

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        side = None
        if (x.B * x.H * x.W <= self.CONCURRENT_MAX_PIX and os.environ.get("LIC_CONCURRENT_RU", "0") == "1" and
                "wnsa" not in os.environ.get("LIC_DEBUG_SERIAL", "")):
            ss = self.__dict__.setdefault("_lic_streams", {})
            if str(x.t.device) not in ss:
                ss[str(x.t.device)] = torch.cuda.Stream(device=x.t.device)
            side = ss[str(x.t.device)]
        main = torch.cuda.current_stream(x.t.device)
        a = x
        if side is not None:   # joined before conv_b's last launch, which reads a
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for blk in self.conv_a:
                    a = blk.run(a)
        else:
            for blk in self.conv_a:
                a = blk.run(a)
        b = self.conv_b[0].run(x)
        b = self.conv_b[1].run(b)
        b = self.conv_b[2].run(b)
        b = self.conv_b[3].run(b)
        b = self.conv_b[4].run(b)
        b = self.conv_b[5].run(b)
        b = self.conv_b[6].run(b)
        b = self.conv_b[7].run(b)
        b = self.conv_b[8].run(b)
        if side is not None:
            main.wait_stream(side)
        return self.conv_b[9].run(b, out, gate_a=a, gate_r=x)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()
