"""CPU oracle — a restatement of the reference's encode -> quantize -> decode path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``lic_amd``) never imports it.

What it is
----------
The reference (xiaobucc/learning-driven-image-compression-algorithm) is itself
PyTorch.  This file restates every function on the hot path as plain fp32
``torch`` CPU ops (ATen/oneDNN conv2d, erfc, log, softmax, layer_norm) **in the
reference's op order**, reading parameters from a ``state_dict``-shaped dict whose
keys are the reference's own module paths.  Each function cites the reference
file:line it follows.  Third-party pieces that the reference imports but does not
vendor (compressai ``ResidualBlock``, ``ResidualBlockWithStride``,
``AttentionBlock``, ``GaussianConditional``, ``EntropyBottleneck._get_medians``,
``subpel_conv3x3``; timm ``DropPath`` = identity at p=0) are restated from
compressai 1.2.x's published source (the version implied by ``_get_medians``;
the reference pins none).

Parity status: **parity unpinned.**  The reference cannot be imported or run in
this environment (missing compressai/timm/torchvision and three in-repo modules,
and a binding permission denial recorded in SURVEY.md section 8(c)); it ships no
tests, fixtures or checkpoints.  This oracle is therefore pinned only by the
analytic known-answer tests in ``tests/test_oracle.py`` (GDN with Gamma=0, WBA
with zero weights, window partition bijection, likelihood normalisation,
ties-to-even rounding, NonNegativeParametrizer round trip of
``ops/parametrizers.py:52-58``) and by the committed golden fixtures it generated
(``tests/golden/``, made by ``tests/golden/make_golden.py``).

Unpinned choice: ``model/DepthwiseSeparableConv.py`` is missing from the reference
(imported at ``net_ga.py:45``, used by ``Syntax_Model`` ``net_ga.py:613-619``).  It is
restated as depthwise 3x3 (groups=C, pad 1, bias) + pointwise 1x1 (bias) with
parameter names ``depthwise`` / ``pointwise``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor
Params = Dict[str, Tensor]


# --------------------------------------------------------------------------- helpers
def _conv(x: Tensor, P: Params, pfx: str, stride: int = 1, padding: int = 0, groups: int = 1) -> Tensor:
    return F.conv2d(x, P[pfx + ".weight"], P.get(pfx + ".bias"), stride, padding, 1, groups)


def _convT(x: Tensor, P: Params, pfx: str, stride: int, padding: int, output_padding: int) -> Tensor:
    return F.conv_transpose2d(x, P[pfx + ".weight"], P.get(pfx + ".bias"), stride, padding, output_padding)


def _linear(x: Tensor, P: Params, pfx: str) -> Tensor:
    return F.linear(x, P[pfx + ".weight"], P.get(pfx + ".bias"))


def gelu(x: Tensor) -> Tensor:  # nn.GELU() default (exact erf form)
    return F.gelu(x)


def lrelu(x: Tensor, slope: float = 0.01) -> Tensor:  # nn.LeakyReLU default slope 0.01
    return F.leaky_relu(x, slope)


# --------------------------------------------------------------------------- ops/
def lower_bound(x: Tensor, bound: Tensor) -> Tensor:
    """ops/bound_ops.py:40-41 (forward): torch.max(x, bound)."""
    return torch.max(x, bound)


def nnp_forward(x: Tensor, bound: Tensor, pedestal: Tensor) -> Tensor:
    """NonNegativeParametrizer.forward, ops/parametrizers.py:48-51."""
    out = lower_bound(x, bound)
    return out ** 2 - pedestal


def nnp_init(x: Tensor, pedestal: Tensor) -> Tensor:
    """NonNegativeParametrizer.init, ops/parametrizers.py:45-46."""
    return torch.sqrt(torch.max(x + pedestal, pedestal))


def ste_round(x: Tensor) -> Tensor:
    """ops/ops.py:34 and net_ga.py:713-719 (forward value)."""
    return torch.round(x) - x.detach() + x


# --------------------------------------------------------------------------- GDN
def gdn_compressai(x: Tensor, P: Params, pfx: str, inverse: bool = False) -> Tensor:
    """layers/gdn.py:62-75 (== compressai GDN used inside ResidualBlockWithStride)."""
    C = x.shape[1]
    beta = nnp_forward(P[pfx + ".beta"], P[pfx + ".beta_reparam.lower_bound.bound"], P[pfx + ".beta_reparam.pedestal"])
    gamma = nnp_forward(P[pfx + ".gamma"], P[pfx + ".gamma_reparam.lower_bound.bound"], P[pfx + ".gamma_reparam.pedestal"])
    gamma = gamma.reshape(C, C, 1, 1)
    norm = F.conv2d(x ** 2, gamma, beta)
    norm = torch.sqrt(norm) if inverse else torch.rsqrt(norm)
    return x * norm


def gdn_model_bounds(P: Params, pfx: str, beta_min: float = 1e-6) -> Tuple[Tensor, Tensor, Tensor]:
    """model/gdn.py:50-55: pedestal = reparam_offset**2 (buffer); beta_bound =
    (beta_min + pedestal)**.5 evaluated in fp32 tensor arithmetic; gamma_bound =
    reparam_offset."""
    reparam_offset = P[pfx + ".reparam_offset"]
    pedestal = P[pfx + ".pedestal"]
    beta_bound = (beta_min + (reparam_offset ** 2)) ** .5
    gamma_bound = reparam_offset
    return pedestal, beta_bound, gamma_bound


def gdn_model(x: Tensor, P: Params, pfx: str, inverse: bool = False) -> Tensor:
    """model/gdn.py:69-92 (GDN: x / sqrt(n)) and :134-156 (IGDN: x * sqrt(n)).
    LowerBound (:11-28) materialises ones(size)*bound and takes torch.max."""
    C = x.shape[1]
    pedestal, beta_bound, gamma_bound = gdn_model_bounds(P, pfx)
    beta_p = P[pfx + ".beta"]
    gamma_p = P[pfx + ".gamma"]
    beta = torch.max(beta_p, torch.ones(beta_p.size()) * beta_bound)
    beta = beta ** 2 - pedestal
    gamma = torch.max(gamma_p, torch.ones(gamma_p.size()) * gamma_bound)
    gamma = gamma ** 2 - pedestal
    gamma = gamma.view(C, C, 1, 1)
    norm_ = F.conv2d(x ** 2, gamma, beta)
    norm_ = torch.sqrt(norm_)
    return x * norm_ if inverse else x / norm_


# --------------------------------------------------------------------------- compressai blocks
def residual_block(x: Tensor, P: Params, pfx: str) -> Tensor:
    """compressai.layers.ResidualBlock (in == out): conv3x3, LReLU, conv3x3, LReLU, +x.
    Used by layers/layers.py:87-102."""
    identity = x
    out = _conv(x, P, pfx + ".conv1", 1, 1)
    out = lrelu(out)
    out = _conv(out, P, pfx + ".conv2", 1, 1)
    out = lrelu(out)
    if (pfx + ".skip.weight") in P:
        identity = _conv(x, P, pfx + ".skip")
    return out + identity


def residual_block_with_stride(x: Tensor, P: Params, pfx: str, stride: int = 2) -> Tensor:
    """compressai.layers.ResidualBlockWithStride (net_ga.py:271,295): conv3x3 s2, LReLU,
    conv3x3, compressai GDN, + conv1x1 s2 skip."""
    identity = x
    out = _conv(x, P, pfx + ".conv1", stride, 1)
    out = lrelu(out)
    out = _conv(out, P, pfx + ".conv2", 1, 1)
    out = gdn_compressai(out, P, pfx + ".gdn")
    if (pfx + ".skip.weight") in P:
        identity = _conv(x, P, pfx + ".skip", stride, 0)
    out = out + identity
    return out


def residual_unit(x: Tensor, P: Params, pfx: str) -> Tensor:
    """compressai AttentionBlock.ResidualUnit: 1x1(N->N/2) ReLU 3x3 ReLU 1x1(->N), +x, ReLU."""
    identity = x
    out = _conv(x, P, pfx + ".conv.0")
    out = F.relu(out)
    out = _conv(out, P, pfx + ".conv.2", 1, 1)
    out = F.relu(out)
    out = _conv(out, P, pfx + ".conv.4")
    out = out + identity
    return F.relu(out)


# --------------------------------------------------------------------------- net_ga blocks
def residual_bottleneck(x: Tensor, P: Params, pfx: str) -> Tensor:
    """net_ga.py:89-103: x + 1x1(N->N/2) GELU 3x3 GELU 1x1(->N)."""
    b = _conv(x, P, pfx + ".branch.0")
    b = gelu(b)
    b = _conv(b, P, pfx + ".branch.2", 1, 1)
    b = gelu(b)
    b = _conv(b, P, pfx + ".branch.4")
    return x + b


# --------------------------------------------------------------------------- window attention (layers/win_attention.py)
def window_partition(x: Tensor, ws: int) -> Tensor:
    """layers/win_attention.py:6-19."""
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, ws, ws, C)


def window_reverse(windows: Tensor, ws: int, H: int, W: int) -> Tensor:
    """layers/win_attention.py:22-35."""
    B = int(windows.shape[0] / (H * W / ws / ws))
    x = windows.view(B, H // ws, W // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, H, W, -1)


def relative_position_index(ws: int) -> Tensor:
    """layers/win_attention.py:64-75."""
    coords = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(ws)], indexing="ij"))
    cf = torch.flatten(coords, 1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1)


def window_attention(x: Tensor, P: Params, pfx: str, ws: int, heads: int, mask) -> Tensor:
    """WindowAttention.forward, layers/win_attention.py:85-116."""
    B_, N, C = x.shape
    qkv = _linear(x, P, pfx + ".qkv").reshape(B_, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4).contiguous()
    q, k, v = qkv[0], qkv[1], qkv[2]
    scale = (C // heads) ** -0.5
    q = q * scale
    attn = q @ k.transpose(-2, -1)
    rpi = relative_position_index(ws)
    table = P[pfx + ".relative_position_bias_table"]
    rpb = table[rpi.view(-1)].view(ws * ws, ws * ws, -1).permute(2, 0, 1).contiguous()
    attn = attn + rpb.unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(B_ // nW, nW, heads, N, N) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, N, N)
    attn = torch.softmax(attn, dim=-1)
    x = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return _linear(x, P, pfx + ".proj")


def wba_mask(H: int, W: int, ws: int, shift: int) -> Tensor:
    """layers/win_attention.py:160-181 (-100 across regions)."""
    img_mask = torch.zeros((1, H, W, 1))
    h_slices = (slice(0, -ws), slice(-ws, -shift), slice(-shift, None))
    w_slices = (slice(0, -ws), slice(-ws, -shift), slice(-shift, None))
    cnt = 0
    for h in h_slices:
        for w in w_slices:
            img_mask[:, h, w, :] = cnt
            cnt += 1
    mw = window_partition(img_mask, ws).view(-1, ws * ws)
    am = mw.unsqueeze(1) - mw.unsqueeze(2)
    return am.masked_fill(am != 0, float(-100.0)).masked_fill(am == 0, float(0.0))


def win_based_attention(x: Tensor, P: Params, pfx: str, heads: int, ws: int, shift: int) -> Tensor:
    """WinBasedAttention.forward, layers/win_attention.py:154-209 (NCHW in/out)."""
    B, C, H, W = x.shape
    shortcut = x
    x = x.permute(0, 2, 3, 1)
    mask = wba_mask(H, W, ws, shift) if shift > 0 else None
    shifted = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2)) if shift > 0 else x
    xw = window_partition(shifted, ws).view(-1, ws * ws, C)
    aw = window_attention(xw, P, pfx + ".attn", ws, heads, mask)
    aw = aw.view(-1, ws, ws, C)
    shifted = window_reverse(aw, ws, H, W)
    x = torch.roll(shifted, shifts=(shift, shift), dims=(1, 2)) if shift > 0 else shifted
    x = x.permute(0, 3, 1, 2).contiguous()
    return shortcut + x


def win_noshift_attention(x: Tensor, P: Params, pfx: str, heads: int, ws: int, shift: int) -> Tensor:
    """Win_noShift_Attention.forward, layers/layers.py:56-111."""
    identity = x
    a = x
    for i in range(3):
        a = residual_block(a, P, f"{pfx}.conv_a.{i}")
    b = win_based_attention(x, P, pfx + ".conv_b.0", heads, ws, shift)
    b = _conv(b, P, pfx + ".conv_b.1")
    b = win_based_attention(b, P, pfx + ".conv_b.2", heads, ws, shift)
    b = residual_block(b, P, pfx + ".conv_b.3")
    b = _conv(b, P, pfx + ".conv_b.4", 1, 1)
    b = win_based_attention(b, P, pfx + ".conv_b.5", heads, ws, shift)
    b = residual_block(b, P, pfx + ".conv_b.6")
    b = _conv(b, P, pfx + ".conv_b.7", 1, 3)
    b = win_based_attention(b, P, pfx + ".conv_b.8", heads, ws, shift)
    b = residual_block(b, P, pfx + ".conv_b.9")
    out = a * torch.sigmoid(b)
    out = out + identity
    return out


# --------------------------------------------------------------------------- WMSA / Swin (Block_unet.py, net_ga.py)
def wmsa_mask(hw: int, ww: int, p: int, shift: int) -> Tensor:
    """WMSA.generate_mask, model/Block_unet.py:197-214 (True -> -inf)."""
    m = torch.zeros(hw, ww, p, p, p, p, dtype=torch.bool)
    s = p - shift
    m[-1, :, :s, :, s:, :] = True
    m[-1, :, s:, :, :s, :] = True
    m[:, -1, :, :s, :, s:] = True
    m[:, -1, :, s:, :, :s] = True
    return m.reshape(hw * ww, p * p, p * p)


def wmsa(x: Tensor, P: Params, pfx: str, head_dim: int, ws: int, type_: str) -> Tensor:
    """WMSA.forward, model/Block_unet.py:216-252. x: [b, h, w, c]."""
    if type_ != "W":
        x = torch.roll(x, shifts=(-(ws // 2), -(ws // 2)), dims=(1, 2))
    b, H, W, c = x.shape
    hw, ww = H // ws, W // ws
    x = x.view(b, hw, ws, ww, ws, c).permute(0, 1, 3, 2, 4, 5).reshape(b, hw * ww, ws * ws, c)
    qkv = _linear(x, P, pfx + ".embedding_layer")
    nh = c // head_dim
    # 'b nw np (threeh c) -> threeh b nw np c'
    qkv = qkv.view(b, hw * ww, ws * ws, 3 * nh, head_dim).permute(3, 0, 1, 2, 4)
    q, k, v = qkv[:nh], qkv[nh:2 * nh], qkv[2 * nh:]
    sim = torch.einsum("hbwpc,hbwqc->hbwpq", q, k) * (head_dim ** -0.5)
    params = P[pfx + ".relative_position_params"]  # [nh, 2ws-1, 2ws-1]
    cord = torch.tensor(np.array([[i, j] for i in range(ws) for j in range(ws)]))
    rel = cord[:, None, :] - cord[None, :, :] + ws - 1
    rpe = params[:, rel[:, :, 0].long(), rel[:, :, 1].long()]
    sim = sim + rpe.unsqueeze(1).unsqueeze(1)
    if type_ != "W":
        m = wmsa_mask(hw, ww, ws, ws // 2)
        sim = sim.masked_fill(m.unsqueeze(0).unsqueeze(0), float("-inf"))
    probs = torch.softmax(sim, dim=-1)
    out = torch.einsum("hbwij,hbwjc->hbwic", probs, v)
    out = out.permute(1, 2, 3, 0, 4).reshape(b, hw * ww, ws * ws, nh * head_dim)
    out = _linear(out, P, pfx + ".linear")
    out = out.view(b, hw, ww, ws, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(b, H, W, -1)
    if type_ != "W":
        out = torch.roll(out, shifts=(ws // 2, ws // 2), dims=(1, 2))
    return out


def block_1(x: Tensor, P: Params, pfx: str, head_dim: int, ws: int, type_: str) -> Tensor:
    """Block_1.forward, net_ga.py:106-128 (LN eps 1e-5)."""
    C = x.shape[-1]
    y = F.layer_norm(x, (C,), P[pfx + ".ln1.weight"], P[pfx + ".ln1.bias"])
    x = x + wmsa(y, P, pfx + ".msa", head_dim, ws, type_)
    y = F.layer_norm(x, (C,), P[pfx + ".ln2.weight"], P[pfx + ".ln2.bias"])
    y = _linear(y, P, pfx + ".mlp.0")
    y = gelu(y)
    y = _linear(y, P, pfx + ".mlp.2")
    return x + y


def swin_block(x: Tensor, P: Params, pfx: str, head_dim: int, ws: int) -> Tensor:
    """SwinBlock.forward, net_ga.py:131-150 (pads when a side <= ws; `resize`
    stays False so the padded map is returned, as in the reference)."""
    if x.size(-1) <= ws or x.size(-2) <= ws:
        pr = (ws - x.size(-2)) // 2
        pc = (ws - x.size(-1)) // 2
        x = F.pad(x, (pc, pc + 1, pr, pr + 1))
    t = x.permute(0, 2, 3, 1)
    t = block_1(t, P, pfx + ".block_1", head_dim, ws, "W")
    t = block_1(t, P, pfx + ".block_2", head_dim, ws, "SW")
    return t.permute(0, 3, 1, 2)


def swatten(x: Tensor, P: Params, pfx: str, head_dim: int = 16, ws: int = 8) -> Tensor:
    """SWAtten.forward, net_ga.py:153-174 (AttentionBlock N=inter_dim=128)."""
    x = _conv(x, P, pfx + ".in_conv")
    identity = x
    z = swin_block(x, P, pfx + ".non_local_block", head_dim, ws)
    a = x
    for i in range(3):
        a = residual_unit(a, P, f"{pfx}.conv_a.{i}")
    b = z
    for i in range(3):
        b = residual_unit(b, P, f"{pfx}.conv_b.{i}")
    b = _conv(b, P, pfx + ".conv_b.3")
    out = a * torch.sigmoid(b)
    out = out + identity
    return _conv(out, P, pfx + ".out_conv")


# --------------------------------------------------------------------------- transforms
def analysis_transform(x: Tensor, P: Params, pfx: str = "a_model") -> Tensor:
    """analysisTransformModel, net_ga.py:253-309 (== net_unet_ha_hs.py:197-232)."""
    t = pfx + ".transform"
    for i in range(3):
        x = residual_bottleneck(x, P, f"{t}.{i}")
    x = residual_block_with_stride(x, P, f"{t}.3", 2)
    x = gdn_model(x, P, f"{t}.4")
    x = F.pad(x, (1, 2, 1, 2))
    x = _conv(x, P, f"{t}.6", 2, 0)
    x = gdn_model(x, P, f"{t}.7")
    x = win_noshift_attention(x, P, f"{t}.8", 8, 8, 4)
    for i in (9, 10, 11):
        x = residual_bottleneck(x, P, f"{t}.{i}")
    x = residual_block_with_stride(x, P, f"{t}.12", 2)
    x = gdn_model(x, P, f"{t}.13")
    x = F.pad(x, (1, 2, 1, 2))
    x = _conv(x, P, f"{t}.15", 2, 0)
    x = win_noshift_attention(x, P, f"{t}.16", 8, 4, 2)
    return x


def synthesis_transform(x: Tensor, P: Params, pfx: str = "s_model") -> Tensor:
    """synthesisTransformModel, net_ga.py:364-403 (== net_unet_ha_hs.py:287-326)."""
    t = pfx + ".transform"
    x = win_noshift_attention(x, P, f"{t}.0", 8, 4, 2)
    x = F.pad(x, (1, 0, 1, 0))
    x = _convT(x, P, f"{t}.2", 2, 3, 1)
    x = gdn_model(x, P, f"{t}.3", inverse=True)
    x = F.pad(x, (1, 0, 1, 0))
    x = _convT(x, P, f"{t}.5", 2, 3, 1)
    x = gdn_model(x, P, f"{t}.6", inverse=True)
    x = win_noshift_attention(x, P, f"{t}.7", 8, 8, 2)
    x = F.pad(x, (1, 0, 1, 0))
    x = _convT(x, P, f"{t}.9", 2, 3, 1)
    x = gdn_model(x, P, f"{t}.10", inverse=True)
    x = F.pad(x, (1, 0, 1, 0))
    x = _convT(x, P, f"{t}.12", 2, 3, 1)
    x = gdn_model(x, P, f"{t}.13", inverse=True)
    return x


def h_a_ga(x: Tensor, P: Params, pfx: str = "h_a") -> Tensor:
    """net_ga.py:811-821."""
    x = gelu(_conv(x, P, pfx + ".0", 1, 1))
    x = gelu(_conv(x, P, pfx + ".2", 1, 1))
    x = gelu(_conv(x, P, pfx + ".4", 2, 1))
    x = gelu(_conv(x, P, pfx + ".6", 1, 1))
    return _conv(x, P, pfx + ".8", 2, 1)


def h_s_ga(x: Tensor, P: Params, pfx: str) -> Tensor:
    """h_mean_s / h_scale_s, net_ga.py:823-845 (subpel_conv3x3 = conv3x3 + PixelShuffle)."""
    x = gelu(_conv(x, P, pfx + ".0", 1, 1))
    x = gelu(F.pixel_shuffle(_conv(x, P, pfx + ".2.0", 1, 1), 2))
    x = gelu(_conv(x, P, pfx + ".4", 1, 1))
    x = gelu(F.pixel_shuffle(_conv(x, P, pfx + ".6.0", 1, 1), 2))
    return _conv(x, P, pfx + ".8", 1, 1)


def residual_block3_5(x: Tensor, P: Params, pfx: str) -> Tensor:
    """ResidualBlock3_5, model/Block_unet.py:295-332."""
    identity = x
    out = lrelu(_conv(x, P, pfx + ".conv1", 1, 1))
    out = lrelu(_conv(out, P, pfx + ".conv2", 1, 2))
    out = lrelu(_conv(out, P, pfx + ".conv3", 1, 1))
    return out + identity


def residual_block5x5(x: Tensor, P: Params, pfx: str) -> Tensor:
    """ResidualBlock5x5, model/Block_unet.py:335-364 (only conv2 is used)."""
    out = lrelu(_conv(x, P, pfx + ".conv2", 1, 2))
    return out + x


def residual_block3x3(x: Tensor, P: Params, pfx: str) -> Tensor:
    """ResidualBlock3x3, model/Block_unet.py:367-398."""
    out = lrelu(_conv(x, P, pfx + ".conv1", 1, 1))
    out = lrelu(_conv(out, P, pfx + ".conv3", 1, 1))
    return out + x


def unet_ha_new(x: Tensor, P: Params, pfx: str = "h_a"):
    """Unet_ha_new.forward, model/Block_unet.py:815-838 (num_heads 8)."""
    C = x.shape[1]
    trans_down_x, conv_down_x = torch.split(x, (C // 2, C // 2), dim=1)
    conv_down_x1 = residual_block3_5(conv_down_x, P, pfx + ".conv1")
    trans_down_x1 = win_based_attention(trans_down_x, P, pfx + ".SpatialTransformer1", 8, 4, 2)
    down_x1 = _conv(torch.cat((conv_down_x1, trans_down_x1), 1), P, pfx + ".down0")
    down_x1 = down_x1 + x
    down_x1 = gelu(_conv(down_x1, P, pfx + ".down1", 2, 1))
    conv_down_y, trans_down_y = torch.split(down_x1, (128, 128), dim=1)
    conv_down_y1 = residual_block5x5(conv_down_y, P, pfx + ".conv2")
    trans_down_y1 = win_based_attention(trans_down_y, P, pfx + ".SpatialTransformer2", 8, 4, 2)
    down_x2 = _conv(torch.cat((conv_down_y1, trans_down_y1), 1), P, pfx + ".down3")
    down_x2 = down_x2 + down_x1
    down_x2 = gelu(_conv(down_x2, P, pfx + ".down2", 2, 1))
    m = residual_bottleneck(down_x2, P, pfx + ".middle.0")
    m = win_based_attention(m, P, pfx + ".middle.1", 8, 2, 1)
    m = residual_bottleneck(m, P, pfx + ".middle.2")
    return m, m, down_x1, x


def unet_hs_new(middle_x: Tensor, down_x1: Tensor, inp: Tensor, P: Params, pfx: str = "h_s") -> Tensor:
    """Unet_hs_new.forward, model/Block_unet.py:868-890 (the `x` argument is unused)."""
    trans_up_x, conv_up_x = torch.split(middle_x, (256, 256), dim=1)
    conv_up_x1 = residual_block3x3(conv_up_x, P, pfx + ".conv3")
    trans_up_x1 = win_based_attention(trans_up_x, P, pfx + ".SpatialTransformer3", 8, 2, 1)
    up_x1 = _conv(torch.cat((conv_up_x1, trans_up_x1), 1), P, pfx + ".up0")
    up_x1 = up_x1 + middle_x
    up_x1 = gelu(_convT(up_x1, P, pfx + ".up1", 2, 2, 1))
    up_x1 = torch.cat((up_x1, down_x1), 1)
    up_x1 = gelu(_convT(up_x1, P, pfx + ".up3", 1, 0, 0))
    conv_up_y, trans_up_y = torch.split(up_x1, (128, 128), dim=1)
    conv_up_y1 = residual_block3x3(conv_up_y, P, pfx + ".conv4")
    trans_up_y1 = win_based_attention(trans_up_y, P, pfx + ".SpatialTransformer2", 8, 2, 1)
    up_x2 = _conv(torch.cat((conv_up_y1, trans_up_y1), 1), P, pfx + ".up5")
    up_x2 = up_x2 + up_x1
    up_x2 = gelu(_convT(up_x2, P, pfx + ".up2", 2, 2, 1))
    up_x2 = torch.cat((up_x2, inp), 1)
    return _convT(up_x2, P, pfx + ".up4", 1, 0, 0)


# --------------------------------------------------------------------------- entropy model / rate
def gaussian_likelihood(values_in: Tensor, scales: Tensor, means: Tensor,
                        scale_bound: float = 0.11, likelihood_bound: float = 1e-9) -> Tensor:
    """compressai GaussianConditional._likelihood + likelihood_lower_bound
    (called at net_ga.py:1049). Phi(t) = 0.5*erfc(-(2**-0.5) t)."""
    half = float(0.5)
    values = values_in - means
    scales = torch.max(scales, torch.tensor([scale_bound], dtype=torch.float32))
    values = torch.abs(values)
    const = float(-(2 ** -0.5))
    upper = half * torch.erfc(const * ((half - values) / scales))
    lower = half * torch.erfc(const * ((-half - values) / scales))
    likelihood = upper - lower
    return torch.max(likelihood, torch.tensor([likelihood_bound], dtype=torch.float32))


def quantize_dequantize(y: Tensor, mu: Tensor) -> Tensor:
    """compressai GaussianConditional.quantize(mode='dequantize'): round(y - mu) + mu."""
    out = y.clone()
    out -= mu
    out = torch.round(out)
    out += mu
    return out


def symbols(y: Tensor, mu: Tensor) -> Tensor:
    """Quantized symbol indices: round_half_even(y - mu) as int32 (compressai 'symbols')."""
    return torch.round(y - mu).to(torch.int32)


# --------------------------------------------------------------------------- syntax head
def depthwise_separable(x: Tensor, P: Params, pfx: str) -> Tensor:
    """Restatement of the missing model/DepthwiseSeparableConv.py (UNPINNED)."""
    C = x.shape[1]
    x = _conv(x, P, pfx + ".depthwise", 1, 1, groups=C)
    return _conv(x, P, pfx + ".pointwise")


def syntax_model(s: Tensor, P: Params, pfx: str = "syntax_model") -> Tensor:
    """Syntax_Model.forward, net_ga.py:626-647."""
    pool = lambda t: F.adaptive_avg_pool2d(t, 1)
    out1 = pool(s)
    d1 = depthwise_separable(s, P, pfx + ".Depth_down0")
    ds1 = F.relu(_conv(d1, P, pfx + ".down0", 2, 1))
    out2 = pool(ds1)
    d2 = depthwise_separable(ds1, P, pfx + ".Depth_down1")
    ds2 = F.relu(_conv(d2, P, pfx + ".down1", 2, 1))
    ds2 = win_noshift_attention(ds2, P, pfx + ".WAM", 8, 4, 2)
    out3 = pool(ds2)
    d3 = depthwise_separable(ds2, P, pfx + ".Depth_down2")
    ds3 = F.relu(_conv(d3, P, pfx + ".down2", 2, 1))
    out4 = pool(ds3)
    out = torch.cat((out1, out2, out3, out4), 1)
    return _conv(out, P, pfx + ".conv")


def conv_generator(x: Tensor, P: Params, pfx: str, out_dim: int) -> Tensor:
    """conv_generator.forward, net_ga.py:597-604 (LeakyReLU 0.2)."""
    b = x.shape[0]
    x = x.view(b, -1)
    x = lrelu(_linear(x, P, pfx + ".transform.0"), 0.2)
    x = lrelu(_linear(x, P, pfx + ".transform.2"), 0.2)
    x = _linear(x, P, pfx + ".transform.4")
    return x.view(b, 3, out_dim, 1, 1)


def batch_conv(weights: Tensor, inputs: Tensor) -> Tensor:
    """Net.batch_conv, net_ga.py:969-979."""
    b, ch, _, _ = inputs.shape
    _, ch_out, _, k, _ = weights.shape
    weights = weights.reshape(b * ch_out, ch, k, k)
    inputs = torch.cat(torch.split(inputs, 1, dim=0), dim=1)
    out = F.conv2d(inputs, weights, stride=1, padding=0, groups=b)
    return torch.cat(torch.split(out, ch_out, dim=1), dim=0)


# --------------------------------------------------------------------------- HAN post-processing (8(f) rank 3)
def han_ca_layer(x: Tensor, P: Params, pfx: str) -> Tensor:
    """CALayer.forward, model/han.py:97-113: x * sigmoid(1x1(relu(1x1(avgpool(x)))))."""
    y = F.adaptive_avg_pool2d(x, 1)
    y = torch.relu(_conv(y, P, pfx + ".conv_du.0"))
    y = torch.sigmoid(_conv(y, P, pfx + ".conv_du.2"))
    return x * y


def han_rcab(x: Tensor, P: Params, pfx: str) -> Tensor:
    """RCAB.forward, model/han.py:205-225 (res_scale unused: res = body(x); res += x)."""
    r = _conv(torch.relu(_conv(x, P, pfx + ".body.0", 1, 1)), P, pfx + ".body.2", 1, 1)
    return han_ca_layer(r, P, pfx + ".body.3") + x


def han_residual_group(x: Tensor, P: Params, pfx: str, n_resblocks: int) -> Tensor:
    """ResidualGroup.forward, model/han.py:228-242."""
    res = x
    for i in range(n_resblocks):
        res = han_rcab(res, P, f"{pfx}.body.{i}")
    res = _conv(res, P, f"{pfx}.body.{n_resblocks}", 1, 1)
    return res + x


def han_lam(x: Tensor, gamma: Tensor) -> Tensor:
    """LAM_Module.forward, model/han.py:124-150 (x: B x N x C x H x W)."""
    B, N, C, H, W = x.size()
    q = x.view(B, N, -1)
    k = x.view(B, N, -1).permute(0, 2, 1)
    energy = torch.bmm(q, k)
    energy_new = torch.max(energy, -1, keepdim=True)[0].expand_as(energy) - energy
    attention = torch.softmax(energy_new, dim=-1)
    out = torch.bmm(attention, x.view(B, N, -1)).view(B, N, C, H, W)
    out = gamma * out + x
    return out.view(B, -1, H, W)


def han_csam(x: Tensor, P: Params, pfx: str) -> Tensor:
    """CSAM_Module.forward, model/han.py:152-188: x * (gamma * sigmoid(conv3d(x))) + x."""
    B, C, H, W = x.size()
    out = torch.sigmoid(F.conv3d(x.unsqueeze(1), P[pfx + ".conv.weight"], P[pfx + ".conv.bias"], 1, 1))
    out = P[pfx + ".gamma"] * out
    out = out.view(B, -1, H, W)
    return x * out + x


def han_head(x: Tensor, P: Params, pfx: str = "HAN", is_high: bool = False) -> Tensor:
    """HAN_Head.forward, model/han.py:247-284."""
    n_rg, n_rb = (6, 12) if is_high else (4, 8)
    x = _conv(x, P, pfx + ".sub_mean")
    x = _conv(x, P, pfx + ".head.0", 1, 1)
    res = x
    res1 = None
    for i in range(n_rg + 1):
        res = (han_residual_group(res, P, f"{pfx}.body.{i}", n_rb) if i < n_rg
               else _conv(res, P, f"{pfx}.body.{i}", 1, 1))
        res1 = res.unsqueeze(1) if res1 is None else torch.cat([res.unsqueeze(1), res1], 1)
    out1 = res
    res = han_lam(res1, P[pfx + ".la.gamma"])
    out2 = _conv(res, P, pfx + ".last_conv", 1, 1)
    out1 = han_csam(out1, P, pfx + ".csa")
    out = torch.cat([out1, out2], 1)
    res = _conv(out, P, pfx + ".last", 1, 1)
    return res + x


# --------------------------------------------------------------------------- full forward
def counter_noise(seed: int, shape_nhwc) -> Tensor:
    """U(-1/2, 1/2) of the seeded-noise rate (liblic's counter hash of (seed, NHWC element
    index), train.hip noise_u): restated in numpy.  The reference draws the same
    distribution from torch's RNG (compressai GaussianConditional 'noise' quantize), so the
    stream itself is the build's own choice -- parity of this mode is pinned on it."""
    n = int(np.prod(shape_nhwc))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        z = np.array([seed], dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + i
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0) - np.float32(0.5)
    return torch.from_numpy(u).view(*shape_nhwc)


def slice_loop(z3: Tensor, latent_means: Tensor, latent_scales: Tensor, P: Params, num_slices: int = 4,
               noise_seed=None, forced_symbols: Optional[Tensor] = None):
    """Channel-conditional slice loop, net_ga.py:1021-1067 (eval / dequantize semantics, or with
    noise_seed the training-mode GaussianConditional the reference's eval actually runs:
    likelihood of y + U(-1/2, 1/2)).

    forced_symbols ([B, 192, h, w] integers, test use): the quantised integers round(y - mu) are
    replaced by these (y_q = s + mu, y_hat = s + mu + lrp), so the later slices' contexts and every
    likelihood are evaluated on another path's symbols -- the reference's arithmetic conditioned on
    that path's near-tie decisions (tests/parity.check_rate)."""
    y_shape = z3.shape[2:]
    y_slices = z3.chunk(num_slices, 1)
    y_hat_slices: List[Tensor] = []
    lik, mus, scs, syms = [], [], [], []
    for i, y_slice in enumerate(y_slices):
        support = y_hat_slices[:4]
        ms = torch.cat([latent_means] + support, dim=1)
        ms = swatten(ms, P, f"atten_mean.{i}.0")
        mu = _conv(gelu(_conv(gelu(_conv(ms, P, f"cc_mean_transforms.{i}.0", 1, 1)), P,
                                   f"cc_mean_transforms.{i}.2", 1, 1)), P, f"cc_mean_transforms.{i}.4", 1, 1)
        mu = mu[:, :, :y_shape[0], :y_shape[1]]
        ss = torch.cat([latent_scales] + support, dim=1)
        ss = swatten(ss, P, f"atten_scale.{i}.0")
        sc = _conv(gelu(_conv(gelu(_conv(ss, P, f"cc_scale_transforms.{i}.0", 1, 1)), P,
                                   f"cc_scale_transforms.{i}.2", 1, 1)), P, f"cc_scale_transforms.{i}.4", 1, 1)
        sc = sc[:, :, :y_shape[0], :y_shape[1]]
        forced = None
        if forced_symbols is not None:
            c0 = i * y_slice.shape[1]
            forced = forced_symbols[:, c0:c0 + y_slice.shape[1]].to(mu.dtype)
        if forced is not None and noise_seed is None:
            y_q = forced + mu
        elif noise_seed is None:
            y_q = quantize_dequantize(y_slice, mu)
        else:
            B_, C_, H_, W_ = y_slice.shape
            y_q = y_slice + counter_noise(noise_seed * num_slices + i, (B_, H_, W_, C_)).permute(0, 3, 1, 2)
        lik.append(gaussian_likelihood(y_q, sc, mu))
        syms.append(symbols(y_slice, mu) if forced is None else forced_symbols[:, c0:c0 + y_slice.shape[1]].clone())
        y_hat_slice = (ste_round(y_slice - mu) if forced is None else forced) + mu
        lrp_support = torch.cat([ms, y_hat_slice], dim=1)
        lrp = _conv(gelu(_conv(gelu(_conv(lrp_support, P, f"lrp_transforms.{i}.0", 1, 1)), P,
                                    f"lrp_transforms.{i}.2", 1, 1)), P, f"lrp_transforms.{i}.4", 1, 1)
        lrp = 0.5 * torch.tanh(lrp)
        y_hat_slice = y_hat_slice + lrp
        y_hat_slices.append(y_hat_slice)
        mus.append(mu)
        scs.append(sc)
    return (torch.cat(y_hat_slices, 1), torch.cat(lik, 1), torch.cat(syms, 1),
            torch.cat(mus, 1), torch.cat(scs, 1))


@torch.no_grad()
def net_forward(x: Tensor, P: Params, arch: str = "net_ga", train_hw=None, M: int = 16,
                post_processing: bool = False, is_high: bool = False, noise_seed=None) -> Dict[str, Tensor]:
    """Net.forward(inputs, 'test') for arch in {'net_ga', 'net_unet_ha_hs'}:
    net_ga.py:981-1144 / net_unet_ha_hs.py:868-1032, eval (dequantize) semantics,
    visualisation / PNG side effects omitted.  Returns a dict of intermediates."""
    B, _, H, W = x.shape
    h, w = train_hw if train_hw is not None else (H, W)
    z3 = analysis_transform(x, P)
    if arch == "net_ga":
        z = h_a_ga(z3, P)
        med = P["entropy_bottleneck.quantiles"][:, :, 1:2]
        z_hat = ste_round(z - med) + med
        latent_scales = h_s_ga(z_hat, P, "h_scale_s")
        latent_means = h_s_ga(z_hat, P, "h_mean_s")
    elif arch == "net_unet_ha_hs":
        z, middle_x, down_x1, inp = unet_ha_new(z3, P)
        med = P["entropy_bottleneck.quantiles"][:, :, 1:2]
        z_hat = ste_round(z - med) + med
        latent_scales = unet_hs_new(middle_x, down_x1, inp, P)
        latent_means = unet_hs_new(middle_x, down_x1, inp, P)
    else:
        raise ValueError(arch)
    syn = syntax_model(z3[:, :M], P)
    syn_r = torch.round(syn)
    y_hat, lik, syms, mus, scs = slice_loop(z3, latent_means, latent_scales, P, noise_seed=noise_seed)
    x_tilde = synthesis_transform(y_hat, P)
    cw = conv_generator(syn_r, P, "conv_weights_gen", M)
    x_bf = torch.tanh(batch_conv(cw, x_tilde))
    if post_processing:                                          # net_ga.py:1096-1100
        x_p = han_head(x_bf, P, "HAN", is_high)
        cw_h = conv_generator(syn_r, P, "conv_weights_gen_HAN", 64)
        x_bf = _conv(batch_conv(cw_h, x_p), P, "add_mean")
    x_t = torch.clamp(x_bf, -1, 1)
    num_pixels = B * h * w
    bpp = torch.sum(torch.log(lik), [0, 1, 2, 3]) / (-np.log(2) * num_pixels)
    gt = torch.round((x + 1) * 127.5)
    x_hat = torch.round(torch.clamp((x_t + 1) * 127.5, 0, 255)).float()
    v_mse = torch.mean((x_hat - gt) ** 2, [1, 2, 3])
    v_psnr = torch.mean(20 * torch.log10(255 / torch.sqrt(v_mse)), 0)
    return dict(z3=z3, z=z, z_hat=z_hat, latent_means=latent_means, latent_scales=latent_scales,
                syntax=syn, y_hat=y_hat, likelihoods=lik, symbols=syms, means=mus, scales=scs,
                x_tilde=x_tilde, x_rec=x_t, bpp=bpp, v_mse=v_mse, v_psnr=v_psnr)


# --------------------------------------------------------------------------- source_net (cfg 1)
def source_net_forward(x: Tensor, P: Params) -> Tensor:
    """source_net.Net.forward returns z right after h_a (source_net.py:846-851):
    a_model = 4x [ZeroPad(1,2,1,2) + conv5x5 s2] with model/gdn GDN between
    (source_net.py:252-278); h_a = abs -> conv3x3 s1 p1, ReLU, conv5x5 s2 p2, ReLU,
    conv5x5 s2 p2 (net_ga.py:440-454 twin, strides [1,2,2])."""
    t = "a_model.transform"
    x = _conv(F.pad(x, (1, 2, 1, 2)), P, f"{t}.1", 2, 0)
    x = gdn_model(x, P, f"{t}.2")
    x = _conv(F.pad(x, (1, 2, 1, 2)), P, f"{t}.4", 2, 0)
    x = gdn_model(x, P, f"{t}.5")
    x = _conv(F.pad(x, (1, 2, 1, 2)), P, f"{t}.7", 2, 0)
    x = gdn_model(x, P, f"{t}.8")
    z3 = _conv(F.pad(x, (1, 2, 1, 2)), P, f"{t}.10", 2, 0)
    h = torch.abs(z3)
    h = F.relu(_conv(h, P, "h_a.transform.0", 1, 1))
    h = F.relu(_conv(h, P, "h_a.transform.2", 2, 2))
    return _conv(h, P, "h_a.transform.4", 2, 2)
