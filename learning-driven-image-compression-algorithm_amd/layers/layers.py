"""Conv helpers and Win_noShift_Attention (reference layers/layers.py:36-111)."""
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
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

    def run(self, x: Act, out: Optional[Act] = None, fork: bool = False) -> Act:
        """fork=True (the 16x16 latents of the a_model / s_model, called on the capture stream): conv_a runs
        on a side stream forked from the current one and joined before the gate, concurrent with conv_b's
        chain -- both are chains of latency-bound launches there.  One level only: the caller guarantees the
        current stream is the capture stream (a nested fork segfaults in hipGraph capture,
        tools/capture_fork_probe.py)."""
        side = None
        if fork and Fn.fork_enabled():
            main = torch.cuda.current_stream(x.t.device)
            side = Fn.aux_stream(x.t.device, "conv_a")
            side.wait_stream(main)
            with torch.cuda.stream(side):
                a = x
                for blk in self.conv_a:
                    a = blk.run(a)
        else:
            a = x
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
            a.t.record_stream(main)     # allocated on the side stream, read by the gate on this one
        return self.conv_b[9].run(b, out, gate_a=a, gate_r=x)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()
