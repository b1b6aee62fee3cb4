"""Window attention with the reference's parameter names
(layers/win_attention.py:38-209).

WinBasedAttention.run = qkv Linear (1x1 GEMM, lic_conv2d_fwd)
                      -> lic_win_attn_fwd (roll + partition + QK^T*scale + rel-pos bias + -100 mask
                         + softmax + AV + reverse + roll back)
                      -> proj Linear with the shortcut add fused in its epilogue.
"""
import os
from typing import Optional

import torch
import torch.nn as nn

from .. import functional as Fn
from ..functional import Act
from ._conv import Linear

__all__ = ["WindowAttention", "WinBasedAttention", "window_partition", "window_reverse"]

_FUSED = os.environ.get("LIC_FUSED_WBA", "1") != "0"
_FUSED_PROJ = os.environ.get("LIC_FUSED_WBA_PROJ", "0") == "1"
_FUSED16 = os.environ.get("LIC_FUSED_WBA16", "1") != "0"


def window_partition(x, window_size=8):
    """Layout helper kept for API parity (layers/win_attention.py:6-19); the hot path
    never materialises windows (the attention kernel addresses them in place)."""
    B, H, W, C = x.shape
    x = x.view(B, H // window_size, window_size, W // window_size, window_size, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, window_size, window_size, C)


def window_reverse(windows, window_size, H, W):
    B = int(windows.shape[0] / (H * W / window_size / window_size))
    x = windows.view(B, H // window_size, W // window_size, window_size, window_size, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, H, W, -1)


def _trunc_normal_(t, std=0.02):
    # timm trunc_normal_(std, a=-2, b=2): truncation bounds are absolute (+-2)
    with torch.no_grad():
        return nn.init.trunc_normal_(t, mean=0., std=std, a=-2., b=2.)


class WindowAttention(nn.Module):
    def __init__(self, dim=192, window_size=(8, 8), num_heads=8, qkv_bias=True, qk_scale=None, attn_drop=0.,
                 proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = window_size
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        ws = window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * window_size[1] - 1),
                                                                     num_heads))
        coords = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(window_size[1])], indexing="ij"))
        cf = torch.flatten(coords, 1)
        rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
        rel[:, :, 0] += ws - 1
        rel[:, :, 1] += window_size[1] - 1
        rel[:, :, 0] *= 2 * window_size[1] - 1
        self.register_buffer("relative_position_index", rel.sum(-1))
        self.qkv = Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = Linear(dim, dim)
        _trunc_normal_(self.relative_position_bias_table, std=.02)


class WinBasedAttention(nn.Module):
    def __init__(self, dim=192, num_heads=8, window_size=8, shift_size=0, qkv_bias=True, qk_scale=None, drop=0.,
                 attn_drop=0., drop_path=0.):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.attn = WindowAttention(dim, window_size=(window_size, window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)

    def run(self, x: Act, out: Optional[Act] = None, **proj_kw) -> Act:
        """out = x + proj(attention(qkv(x))); extra epilogue kwargs go to the proj launch.  Under fp32x6
        at C = 192 / 8 heads / 8x8 windows the qkv Linear and the attention are one launch
        (Fn.wba_qkv_attn: the 3C qkv map never reaches HBM; bit-identical; LIC_FUSED_WBA=0 for the
        three-launch path).  LIC_FUSED_WBA_PROJ=1 also folds the proj + shortcut into that launch
        (bit-identical, but slower today: DESIGN.md section 5)."""
        if _FUSED and Fn.wba_qkv_attn_ok(x, self.dim, self.num_heads, self.window_size):
            # the fused proj stores 16 B per lane: only into a fresh buffer or a 16-B aligned view
            # with 4-element rows, never onto x (the shortcut) -- else the proj runs as its own launch
            fuse_proj = _FUSED_PROJ and not proj_kw and (
                out is None or (out.t.data_ptr() != x.t.data_ptr() and out.ptr % 16 == 0 and out.ld % 4 == 0))
            a = Fn.wba_qkv_attn(x, self.attn.qkv.packed(x.dtype), self.num_heads, self.window_size, self.shift_size,
                                self.attn.relative_position_bias_table, self.num_heads, 1,
                                1 if self.shift_size > 0 else 0, float(self.attn.scale),
                                out=out if fuse_proj else None,
                                proj_pk=self.attn.proj.packed(x.dtype) if fuse_proj else None)
            return a if fuse_proj else self.attn.proj.run(a, out, r1=x, **proj_kw)
        if _FUSED16 and Fn.wba16_qkv_attn_ok(x, self.dim, self.num_heads, self.window_size):
            # 16-bit: qkv + attention in one launch (csrc/wba16.hip); LIC_FUSED_WBA16=0 for two launches
            a = Fn.wba16_qkv_attn(x, self.attn.qkv.packed(x.dtype), self.num_heads, self.window_size,
                                  self.shift_size, self.attn.relative_position_bias_table, self.num_heads, 1,
                                  1 if self.shift_size > 0 else 0, float(self.attn.scale))
            return self.attn.proj.run(a, out, r1=x, **proj_kw)
        qkv = self.attn.qkv.run(x)
        a = Fn.win_attn(qkv, self.dim, self.num_heads, self.window_size, self.shift_size,
                        self.attn.relative_position_bias_table, self.num_heads, 1,
                        1 if self.shift_size > 0 else 0, False, float(self.attn.scale))
        return self.attn.proj.run(a, out, r1=x, **proj_kw)

    def forward(self, x):
        return self.run(Act.from_nchw(x)).nchw()
