"""HAN post-processing head (reference model/han.py, used at net_ga.py:1096-1100 when
``post_processing=True``), with the reference's class names and state_dict keys.

Every convolution runs on lic_conv2d_fwd (MFMA halo / implicit-GEMM kernels); the
channel attention (CALayer), the layer attention over the stacked group outputs
(LAM_Module) and the 3-D channel-spatial attention (CSAM_Module) run on the glue
kernels of csrc/han.hip.  The group outputs are written straight into the channel
windows of one NHWC buffer in the order LAM reads them (newest first, han.py:266-270),
so the reference's unsqueeze/cat stack is never materialised.
"""
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
from .._ffi import ACT_RELU
from ..functional import Act
from ..layers._conv import Conv2d

__all__ = ["default_conv", "MeanShift", "CALayer", "RCAB", "ResidualGroup", "LAM_Module", "CSAM_Module", "HAN_Head"]


def default_conv(in_channels, out_channels, kernel_size, bias=True) -> Conv2d:
    """han.py:7-10."""
    return Conv2d(in_channels, out_channels, kernel_size, padding=(kernel_size // 2), bias=bias)


class MeanShift(Conv2d):
    """han.py:12-22: 1x1 conv 3->3 with weight eye/std and bias sign*range*mean/std."""

    def __init__(self, rgb_range, rgb_mean=(0.4488, 0.4371, 0.4040), rgb_std=(1.0, 1.0, 1.0), sign=-1):
        super().__init__(3, 3, kernel_size=1)
        std = torch.Tensor(rgb_std)
        self.weight.data = torch.eye(3).view(3, 3, 1, 1) / std.view(3, 1, 1, 1)
        self.bias.data = sign * rgb_range * torch.Tensor(rgb_mean) / std
        for p in self.parameters():
            p.requires_grad = False

    def post_params(self) -> torch.Tensor:
        """fp32 [W (3x3 row-major), b (3)] for lic_recon_fwd's fused 1x1 3->3."""
        return torch.cat([self.weight.detach().float().reshape(9), self.bias.detach().float().reshape(3)]).contiguous()


def _cached(mod: nn.Module, name: str, params, build):
    key = tuple((p.data_ptr(), p._version) for p in params)
    c = mod.__dict__.get(name)
    if c is None or c[0] != key:
        c = (key, build())
        mod.__dict__[name] = c
    return c[1]


class CALayer(nn.Module):
    """han.py:96-113: x * sigmoid(1x1(relu(1x1(avgpool(x)))))."""

    def __init__(self, channel, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.conv_du = nn.Sequential(Conv2d(channel, channel // reduction, 1, padding=0, bias=True),
                                     nn.ReLU(inplace=True),
                                     Conv2d(channel // reduction, channel, 1, padding=0, bias=True),
                                     nn.Sigmoid())

    def _mats(self):
        c1, c2 = self.conv_du[0], self.conv_du[2]
        ps = (c1.weight, c1.bias, c2.weight, c2.bias)
        return _cached(self, "_lic_ca", ps, lambda: tuple(
            p.detach().float().reshape(p.shape[0], -1).contiguous() if p.dim() > 1 else p.detach().float().contiguous()
            for p in ps))

    def run(self, r: Act, x: Act, out: Optional[Act] = None) -> Act:
        """r * y + x (the RCAB residual fused)."""
        # avg_pool in two passes (per-chunk sums, then their sum inside ca_apply)
        nchunk = max(1, min(64, -(-(r.H * r.W) // 1024)))
        parts = torch.empty((r.B * (nchunk + 1) * r.c,), dtype=torch.float32, device=r.t.device)
        Fn.pool_partials(r, nchunk, parts)
        w1, b1, w2, b2 = self._mats()
        return Fn.ca_apply(r, x, parts, nchunk, w1, b1, w2, b2, out)


class RCAB(nn.Module):
    """han.py:191-225: conv3x3, ReLU, conv3x3, CALayer; res += x."""

    def __init__(self, conv, n_feat, kernel_size, reduction, bias=True, bn=False, act=nn.ReLU(True), res_scale=1):
        super().__init__()
        if bn:
            raise NotImplementedError("RCAB(bn=True) is not used by HAN_Head")
        self.body = nn.Sequential(conv(n_feat, n_feat, kernel_size, bias=bias), act,
                                  conv(n_feat, n_feat, kernel_size, bias=bias), CALayer(n_feat, reduction))
        self.res_scale = res_scale

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        t = self.body[0].run(x, act=ACT_RELU)
        r = self.body[2].run(t)
        return self.body[3].run(r, x, out)


class ResidualGroup(nn.Module):
    """han.py:228-242: n RCABs + conv3x3, + x."""

    def __init__(self, conv, n_feat, kernel_size, reduction, act, res_scale, n_resblocks):
        super().__init__()
        mods = [RCAB(conv, n_feat, kernel_size, reduction, bias=True, bn=False, act=nn.ReLU(True), res_scale=1)
                for _ in range(n_resblocks)]
        mods.append(conv(n_feat, n_feat, kernel_size))
        self.body = nn.Sequential(*mods)

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        res = x
        for m in list(self.body)[:-1]:
            res = m.run(res)
        return self.body[-1].run(res, out, r1=x)


class LAM_Module(nn.Module):
    """han.py:115-150 (layer attention over the stacked group outputs)."""

    def __init__(self, in_dim):
        super().__init__()
        self.chanel_in = in_dim
        self.gamma = nn.Parameter(torch.zeros(1))
        self.softmax = nn.Softmax(dim=-1)

    def run(self, stack: Act, ngroups: int, out: Optional[Act] = None) -> Act:
        g = _cached(self, "_lic_g", (self.gamma,), lambda: self.gamma.detach().float().contiguous())
        return Fn.lam(stack, ngroups, g, out)


class CSAM_Module(nn.Module):
    """han.py:152-188 (Conv3d(1, 1, 3, 1, 1) over (channel, y, x), sigmoid, gamma)."""

    def __init__(self, in_dim):
        super().__init__()
        self.chanel_in = in_dim
        self.conv = nn.Conv3d(1, 1, 3, 1, 1)
        self.gamma = nn.Parameter(torch.zeros(1))
        self.sigmoid = nn.Sigmoid()

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        ps = (self.conv.weight, self.conv.bias, self.gamma)
        prm = _cached(self, "_lic_p", ps, lambda: torch.cat([p.detach().float().reshape(-1) for p in ps]).contiguous())
        return Fn.csam(x, prm, out)


class HAN_Head(nn.Module):
    """han.py:244-284."""

    def __init__(self, is_high=False, conv=default_conv):
        super().__init__()
        n_resgroups, n_resblocks = (6, 12) if is_high else (4, 8)
        n_feats, kernel_size, reduction = 64, 3, 32
        act = nn.ReLU(True)
        rgb_mean, rgb_std = (0.4488, 0.4371, 0.4040), (1.0, 1.0, 1.0)
        self.n_resgroups = n_resgroups
        self.n_feats = n_feats
        self.sub_mean = MeanShift(1.0, rgb_mean, rgb_std)
        self.head = nn.Sequential(conv(3, n_feats, kernel_size))
        body = [ResidualGroup(conv, n_feats, kernel_size, reduction, act=act, res_scale=1, n_resblocks=n_resblocks)
                for _ in range(n_resgroups)]
        body.append(conv(n_feats, n_feats, kernel_size))
        self.body = nn.Sequential(*body)
        self.csa = CSAM_Module(n_feats)
        self.la = LAM_Module(n_feats)
        self.last_conv = Conv2d(n_feats * (n_resgroups + 1), n_feats, 3, 1, 1)
        self.last = Conv2d(n_feats * 2, n_feats, 3, 1, 1)

    def run(self, x: Act, out: Optional[Act] = None) -> Act:
        """x: 3-channel view (zero-padded pixels preferred) -> 64-channel Act."""
        B, H, W = x.B, x.H, x.W
        dev, dt = x.t.device, x.dtype
        F_, G = self.n_feats, self.n_resgroups + 1
        epc = 16 // x.t.element_size()
        # sub_mean into a zero-padded 3-channel image so the head conv runs on MFMA
        xm = Act(torch.zeros((B, H, W, epc), dtype=dt, device=dev), 0, 3, epc)
        self.sub_mean.run(x, Act(xm.t, 0, 3))
        head = self.head[0].run(xm)
        # stack[:, window G-1-i] = output of body module i (han.py:266-270: newest first)
        stack = Act.empty(B, H, W, F_ * G, dt, dev)
        res = head
        for i, m in enumerate(self.body):
            win = stack.ch((G - 1 - i) * F_, (G - i) * F_)
            res = m.run(res, win)
        out1 = stack.ch(0, F_)
        lam = self.la.run(stack, G)
        cat = Act.empty(B, H, W, 2 * F_, dt, dev)
        self.last_conv.run(lam, cat.ch(F_, 2 * F_))
        self.csa.run(out1, cat.ch(0, F_))
        return self.last.run(cat, out, r1=head)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()
