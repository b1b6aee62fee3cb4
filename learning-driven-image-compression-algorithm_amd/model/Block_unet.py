"""Blocks of reference model/Block_unet.py used on the hot path: WMSA (Swin MSA of
the slice-loop SWAtten, :170-252), the residual blocks (:295-415) and the
net_unet_ha_hs hyper networks Unet_ha_new / Unet_hs_new (:774-890).
All compute runs on liblic; channel splits / concatenations are channel views.
"""
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
from .._ffi import ACT_GELU, ACT_LRELU
from ..functional import Act
from ..layers._conv import Conv2d, ConvTranspose2d, Linear
from ..layers.win_attention import WinBasedAttention, _trunc_normal_

__all__ = ["WMSA", "ResidualBlock3_5", "ResidualBlock5x5", "ResidualBlock3x3", "ResidualBottleneck",
           "Unet_ha_new", "Unet_hs_new"]


def conv1x1(in_ch, out_ch, stride=1):
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def conv3x3(in_ch, out_ch, stride=1):
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv5x5(in_ch, out_ch, stride=1):
    return Conv2d(in_ch, out_ch, kernel_size=5, stride=stride, padding=2)


class WMSA(nn.Module):
    """Swin window MSA (model/Block_unet.py:170-252): qkv = embedding_layer(x);
    sim = (q k^T) * scale + rel-pos bias; SW type: roll by -ws/2 and -inf mask on
    the last window row/column; softmax; AV; linear.  The residual add of
    Block_1 is fused into the ``linear`` launch (r1)."""

    def __init__(self, input_dim, output_dim, head_dim, window_size, type):
        super().__init__()
        self.input_dim = input_dim
        self.output_dim = output_dim
        self.head_dim = head_dim
        self.scale = self.head_dim ** -0.5
        self.n_heads = input_dim // head_dim
        self.window_size = window_size
        self.type = type
        self.embedding_layer = Linear(self.input_dim, 3 * self.input_dim, bias=True)
        rp = torch.zeros((2 * window_size - 1) * (2 * window_size - 1), self.n_heads)
        _trunc_normal_(rp, std=.02)
        self.linear = Linear(self.input_dim, self.output_dim)
        # [n_heads, 2ws-1, 2ws-1] as in the reference (:192-195)
        self.relative_position_params = nn.Parameter(
            rp.view(2 * window_size - 1, 2 * window_size - 1, self.n_heads).transpose(1, 2).transpose(0, 1))

    def run(self, x: Act, residual: Act, out: Optional[Act] = None) -> Act:
        ws = self.window_size
        qkv = self.embedding_layer.run(x)
        table = self.relative_position_params.contiguous()
        sw = self.type != "W"
        a = Fn.win_attn(qkv, self.input_dim, self.n_heads, ws, ws // 2 if sw else 0, table, 1, (2 * ws - 1) ** 2,
                        2 if sw else 0, True, float(self.scale))
        return self.linear.run(a, out, r1=residual)


class ResidualBottleneck(nn.Module):
    """x + conv1x1(N->N/2) GELU conv3x3 GELU conv1x1(->N) (net_ga.py:89-103, Block_unet.py:401-415)."""

    def __init__(self, N=192, act=nn.GELU):
        super().__init__()
        self.branch = nn.Sequential(conv1x1(N, N // 2), act(),
                                    Conv2d(N // 2, N // 2, kernel_size=3, stride=1, padding=1), act(),
                                    conv1x1(N // 2, N))

    def rb3_ok(self, x: Act) -> bool:
        return x.c == 3 and self.branch[0].out_channels == 1

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        if self.rb3_ok(x) and out is None:
            return Fn.rb3(x, self._rb3_params())                 # whole block in one pass
        t = self.branch[0].run(x, act=ACT_GELU)
        t = self.branch[2].run(t, act=ACT_GELU)
        return self.branch[4].run(t, out, r1=x)

    def _rb3_params(self) -> torch.Tensor:
        b = self.branch
        ps = (b[0].weight, b[0].bias, b[2].weight, b[2].bias, b[4].weight, b[4].bias)
        key = tuple((p.data_ptr(), p._version) for p in ps)
        c = self.__dict__.get("_rb3_cache")
        if c is None or c[0] != key:
            flat = torch.cat([p.detach().float().reshape(-1) for p in ps]).contiguous()
            c = (key, flat)
            self.__dict__["_rb3_cache"] = c
        return c[1]

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()


class ResidualBlock3_5(nn.Module):
    """Block_unet.py:295-332: lrelu(conv3x3) lrelu(conv5x5) lrelu(conv3x3) + x."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv5x5(out_ch, out_ch)
        self.conv3 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        t = self.conv1.run(x, act=ACT_LRELU)
        t = self.conv2.run(t, act=ACT_LRELU)
        identity = self.skip.run(x) if self.skip is not None else x
        return self.conv3.run(t, out, act=ACT_LRELU, r1=identity)


class ResidualBlock5x5(nn.Module):
    """Block_unet.py:335-364: lrelu(conv5x5(x)) + x (conv1 / conv3 unused, kept for state_dict)."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv2 = conv5x5(out_ch, out_ch)
        self.conv3 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        identity = self.skip.run(x) if self.skip is not None else x
        return self.conv2.run(x, out, act=ACT_LRELU, r1=identity)


class ResidualBlock3x3(nn.Module):
    """Block_unet.py:367-398: lrelu(conv3x3) lrelu(conv3x3) + x."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        self.conv1 = conv3x3(in_ch, out_ch)
        self.leaky_relu = nn.LeakyReLU(inplace=True)
        self.conv3 = conv3x3(out_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else None

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        t = self.conv1.run(x, act=ACT_LRELU)
        identity = self.skip.run(x) if self.skip is not None else x
        return self.conv3.run(t, out, act=ACT_LRELU, r1=identity)


class Unet_ha_new(nn.Module):
    """Hyper-analysis of net_unet_ha_hs (Block_unet.py:774-838).  Returns
    (z, middle_x, down_x1, x) like the reference."""

    def __init__(self, inchannels, num_heads, depth):
        super().__init__()
        self.inchannels = inchannels
        self.num_heads = num_heads
        self.depth = depth
        self.SpatialTransformer1 = WinBasedAttention(inchannels // 2, self.num_heads, window_size=4, shift_size=2)
        self.ResBlock1 = ResidualBottleneck(96)
        self.SpatialTransformer2 = WinBasedAttention(128, self.num_heads, window_size=4, shift_size=2)
        self.ResBlock2 = ResidualBottleneck(128)
        self.ResBlock3 = ResidualBottleneck(256)
        self.conv1 = ResidualBlock3_5(inchannels // 2, inchannels // 2)
        self.conv2 = ResidualBlock5x5(128, 128)
        self.down0 = Conv2d(self.inchannels, self.inchannels, 1, 1, 0, bias=True)
        self.down1 = Conv2d(self.inchannels, 256, kernel_size=3, stride=2, padding=1)
        self.down2 = Conv2d(256, 512, kernel_size=3, stride=2, padding=1)
        self.down3 = Conv2d(256, 256, 1, 1, 0, bias=True)
        self.middle = nn.Sequential(ResidualBottleneck(512), WinBasedAttention(512, self.num_heads, window_size=2,
                                                                               shift_size=1), ResidualBottleneck(512))
        self.relu = nn.GELU()

    def run(self, x: Act):
        C = x.c
        h = C // 2
        B, H, W = x.B, x.H, x.W
        cat1 = Act.empty(B, H, W, C, x.dtype, x.t.device)
        self.conv1.run(x.ch(h, C), out=cat1.ch(0, h))              # conv branch on the 2nd half
        self.SpatialTransformer1.run(x.ch(0, h), out=cat1.ch(h, C))  # transformer branch on the 1st half
        d = self.down0.run(cat1, r1=x)
        down_x1 = self.down1.run(d, act=ACT_GELU)
        cat2 = Act.empty(B, down_x1.H, down_x1.W, 256, x.dtype, x.t.device)
        self.conv2.run(down_x1.ch(0, 128), out=cat2.ch(0, 128))
        self.SpatialTransformer2.run(down_x1.ch(128, 256), out=cat2.ch(128, 256))
        d2 = self.down3.run(cat2, r1=down_x1)
        d2 = self.down2.run(d2, act=ACT_GELU)
        m = self.middle[0].run(d2)
        m = self.middle[1].run(m)
        m = self.middle[2].run(m)
        return m, m, down_x1, x


class Unet_hs_new(nn.Module):
    """Hyper-synthesis of net_unet_ha_hs (Block_unet.py:841-890).  Its first argument
    is never read (reference :868); it consumes encoder-side middle_x, down_x1, input."""

    def __init__(self, out_channels, num_heads, depth):
        super().__init__()
        self.out_channels = out_channels
        self.num_heads = num_heads
        self.depth = depth
        self.SpatialTransformer2 = WinBasedAttention(128, self.num_heads, window_size=2, shift_size=1)
        self.SpatialTransformer3 = WinBasedAttention(256, self.num_heads, window_size=2, shift_size=1)
        self.up0 = Conv2d(512, 512, 1, 1, 0, bias=True)
        self.up1 = ConvTranspose2d(512, 256, 5, 2, 2, output_padding=1, bias=True)
        self.up2 = ConvTranspose2d(256, 192, 5, 2, 2, output_padding=1, bias=True)
        self.up3 = ConvTranspose2d(512, 256, 1, 1, 0, bias=True)
        self.up4 = ConvTranspose2d(384, self.out_channels, 1, 1, 0, bias=True)
        self.up5 = Conv2d(256, 256, 1, 1, 0, bias=True)
        self.conv3 = ResidualBlock3x3(256, 256)
        self.conv4 = ResidualBlock3x3(128, 128)
        self.relu = nn.GELU()

    def run(self, x, middle_x: Act, down_x1: Act, inp: Act, out: Optional[Act] = None) -> Act:
        B, dt, dev = middle_x.B, middle_x.dtype, middle_x.t.device
        cat0 = Act.empty(B, middle_x.H, middle_x.W, 512, dt, dev)
        self.conv3.run(middle_x.ch(256, 512), out=cat0.ch(0, 256))
        self.SpatialTransformer3.run(middle_x.ch(0, 256), out=cat0.ch(256, 512))
        u = self.up0.run(cat0, r1=middle_x)
        Ho, Wo = self.up1.out_hw(u.H, u.W)
        cat1 = Act.empty(B, Ho, Wo, 512, dt, dev)
        self.up1.run(u, out=cat1.ch(0, 256), act=ACT_GELU)
        Fn.copy(down_x1, cat1.ch(256, 512))
        u1 = self.up3.run(cat1, act=ACT_GELU)
        cat2 = Act.empty(B, u1.H, u1.W, 256, dt, dev)
        self.conv4.run(u1.ch(0, 128), out=cat2.ch(0, 128))
        self.SpatialTransformer2.run(u1.ch(128, 256), out=cat2.ch(128, 256))
        u2 = self.up5.run(cat2, r1=u1)
        Ho, Wo = self.up2.out_hw(u2.H, u2.W)
        cat3 = Act.empty(B, Ho, Wo, 192 + inp.c, dt, dev)
        self.up2.run(u2, out=cat3.ch(0, 192), act=ACT_GELU)
        Fn.copy(inp, cat3.ch(192, 192 + inp.c))
        return self.up4.run(cat3, out)
