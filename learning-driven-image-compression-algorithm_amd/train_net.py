"""Net.forward(x, 'train') on liblic autograd ops.

The reference trains with ``bpp, mse = net(x, 'train'); loss = lambda*255^2*mse + bpp;
loss.backward()`` (train_net_unet.py:177-196) and finetunes the encoder the same way
(eval_net.py:170-179).  This module walks the same reference-named modules as the
inference path (their parameters, same state_dict) but builds the forward from
``lic_amd.autograd`` Functions, so every forward AND backward op is a liblic launch:
convolutions (dgrad via re-packed forward launches, MFMA split-K wgrad), GDN/IGDN with
the LowerBound gradient rule, window attention / WMSA, LayerNorm, gates, the
training-mode GaussianConditional rate (additive uniform noise, net_ga.py:1049) and the
tanh(batch_conv) reconstruction + nn.MSELoss (net_ga.py:1089-1115).

Activations are NHWC; channel concatenations / slices and PixelShuffle are layout
plumbing (torch views and copies), never arithmetic.

Train-mode semantics (net_ga.py:981-1115, mode == 'train'):
  * GaussianConditional adds U(-1/2, 1/2) noise to y before pricing it; the noise is a
    counter-based hash of (seed, element) generated inside the rate kernels (torch's
    Philox stream cannot be reproduced; the distribution is the same).
  * y_hat_i = ste_round(y_i - mu_i) + mu_i (+ 0.5 tanh(lrp)), z_hat = ste_round(z - m) + m,
    syntax = bypass_round(...) — straight-through gradients.
  * bpp = sum ln L / (-ln 2 * B*h*w) over the y slices (z likelihoods discarded);
    mse = nn.MSELoss()(tanh(batch_conv(W(syntax), g_s(y_hat))), x).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import autograd as AG
from ._ffi import ACT_GELU, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_ROUND
from .layers.gdn import GDN as CompressaiGDN

__all__ = ["net_forward_train", "analysis", "synthesis", "syntax", "generator", "swatten",
           "win_noshift_attention"]


# --------------------------------------------------------------------------- leaf layers
def conv(m, x, act: int = ACT_NONE, slope: float = 0.01, pad=None, residual=None, res_act: bool = False):
    """nn.Conv2d (reference names) on an NHWC tensor; pad overrides the symmetric padding
    (top, left, bottom, right) for the ZeroPad2d + conv pairs.  residual: conv(x) + residual (res_act:
    act(conv(x) + residual)) in the conv's epilogue."""
    if pad is None:
        p = m.padding[0]
        pad = (p, p, p, p)
    if m.groups != 1:
        y = AG.dwconv2d(x, m.weight, m.bias, m.stride[0], pad)
        if residual is not None:
            raise ValueError("conv: no fused residual for depthwise convs")
        return AG.activation(y, act, slope) if act != ACT_NONE else y
    return AG.conv2d(x, m.weight, m.bias, m.stride[0], pad, act, slope, residual=residual, res_act=res_act)


def linear(m, x, act: int = ACT_NONE, slope: float = 0.01, residual=None):
    """nn.Linear over the channels of every pixel (a 1x1 convolution); + residual in its epilogue."""
    return AG.conv2d(x, m.weight[:, :, None, None], m.bias, 1, 0, act, slope, residual=residual)


def conv_t(m, x, prepad=(1, 1)):
    """ZeroPad2d((1, 0, 1, 0)) + nn.ConvTranspose2d(k5, s2, p3, op1) (net_ga.py:373-397)."""
    return AG.conv_transpose2d(x, m.weight, m.bias, m.stride[0], m.padding[0], m.output_padding[0], prepad)


def gdn(m, x):
    """model/gdn.py GDN / IGDN (x / sqrt(n), x * sqrt(n)) or compressai GDN (x * rsqrt(n))."""
    if isinstance(m, CompressaiGDN):
        bb, gb, ped = m._consts
        return AG.gdn(x, m.beta, m.gamma, bb, gb, ped, inverse=m.inverse, rsqrt=True)
    return AG.gdn(x, m.beta, m.gamma, m._beta_bound, m._gamma_bound, m._pedestal, inverse=m._inverse_math)


def pixel_shuffle(x):
    """nn.PixelShuffle(2) in NHWC: channel c*4 + 2i + j of (y, x) -> channel c of (2y+i, 2x+j)."""
    B, h, w, c4 = x.shape
    c = c4 // 4
    return x.view(B, h, w, c, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(B, 2 * h, 2 * w, c)


# --------------------------------------------------------------------------- blocks
def residual_bottleneck(m, x):
    """net_ga.py:89-103: x + 1x1 GELU 3x3 GELU 1x1."""
    b = m.branch
    t = conv(b[0], x, ACT_GELU)
    t = conv(b[2], t, ACT_GELU)
    return conv(b[4], t, residual=x)


def residual_block(m, x):
    """compressai ResidualBlock: lrelu(conv3x3) lrelu(conv3x3) + identity."""
    t = conv(m.conv1, x, ACT_LRELU)
    t = conv(m.conv2, t, ACT_LRELU)
    idn = conv(m.skip, x) if m.skip is not None else x
    return AG.add(t, idn)


def residual_block_with_stride(m, x):
    """compressai ResidualBlockWithStride: conv3x3 s2, lrelu, conv3x3, GDN, + 1x1 s2 skip."""
    t = conv(m.conv1, x, ACT_LRELU)
    t = gdn(m.gdn, conv(m.conv2, t))
    idn = conv(m.skip, x) if m.skip is not None else x
    return AG.add(t, idn)


def residual_unit(m, x):
    """compressai AttentionBlock.ResidualUnit: relu(1x1 relu 3x3 relu 1x1 + x)."""
    c = m.conv
    t = conv(c[0], x, ACT_RELU)
    t = conv(c[2], t, ACT_RELU)
    return conv(c[4], t, ACT_RELU, residual=x, res_act=True)


def wba(m, x):
    """WinBasedAttention (layers/win_attention.py:154-209): x + proj(attn(qkv(x)))."""
    at = m.attn
    qkv = linear(at.qkv, x)
    a = AG.win_attn(qkv, at.relative_position_bias_table, m.dim, m.num_heads, m.window_size, m.shift_size,
                    tab_sr=m.num_heads, tab_sh=1, mask_kind=1 if m.shift_size > 0 else 0, scale_after=False,
                    scale=float(at.scale))
    return linear(at.proj, a, residual=x)


def win_noshift_attention(m, x):
    """Win_noShift_Attention (layers/layers.py:56-111): x + conv_a(x) * sigmoid(conv_b(x))."""
    a = x
    for blk in m.conv_a:
        a = residual_block(blk, a)
    cb = m.conv_b
    b = wba(cb[0], x)
    b = conv(cb[1], b)
    b = wba(cb[2], b)
    b = residual_block(cb[3], b)
    b = conv(cb[4], b)
    b = wba(cb[5], b)
    b = residual_block(cb[6], b)
    b = conv(cb[7], b)
    b = wba(cb[8], b)
    b = residual_block(cb[9], b)
    return AG.gate(b, a, x)


def wmsa(m, x, residual):
    """WMSA (model/Block_unet.py:216-252) + the Block_1 residual."""
    ws = m.window_size
    sw = m.type != "W"
    qkv = linear(m.embedding_layer, x)
    table = m.relative_position_params.contiguous()   # [heads, 2ws-1, 2ws-1]
    a = AG.win_attn(qkv, table, m.input_dim, m.n_heads, ws, ws // 2 if sw else 0, tab_sr=1,
                    tab_sh=(2 * ws - 1) ** 2, mask_kind=2 if sw else 0, scale_after=True, scale=float(m.scale))
    return linear(m.linear, a, residual=residual)


def block_1(m, x):
    """net_ga.py:125-128: x + WMSA(LN(x)); x + MLP(LN(x))."""
    y = AG.layernorm(x, m.ln1.weight, m.ln1.bias, m.ln1.eps)
    x1 = wmsa(m.msa, y, x)
    y = AG.layernorm(x1, m.ln2.weight, m.ln2.bias, m.ln2.eps)
    h = linear(m.mlp[0], y, ACT_GELU)
    return linear(m.mlp[2], h, residual=x1)


def swin_block(m, x):
    """net_ga.py:138-150 (pads a latent whose side <= ws and returns the padded map)."""
    ws = m.window_size
    if x.shape[1] <= ws or x.shape[2] <= ws:
        pr, pc = (ws - x.shape[1]) // 2, (ws - x.shape[2]) // 2
        x = F.pad(x, (0, 0, pc, pc + 1, pr, pr + 1))
    return block_1(m.block_2, block_1(m.block_1, x))


def swatten(m, x):
    """SWAtten (net_ga.py:153-174)."""
    x = conv(m.in_conv, x)
    z = swin_block(m.non_local_block, x)
    a = x
    for u in m.conv_a:
        a = residual_unit(u, a)
    b = z
    for u in list(m.conv_b)[:3]:
        b = residual_unit(u, b)
    b = conv(m.conv_b[3], b)
    return conv(m.out_conv, AG.gate(b, a, x))


# --------------------------------------------------------------------------- transforms
def analysis(m, x):
    """analysisTransformModel (net_ga.py:253-309)."""
    t = m.transform
    for i in range(3):
        x = residual_bottleneck(t[i], x)
    x = gdn(t[4], residual_block_with_stride(t[3], x))
    x = gdn(t[7], conv(t[6], x, pad=(1, 1, 2, 2)))     # ZeroPad2d((1, 2, 1, 2)) + conv5x5 s2
    x = win_noshift_attention(t[8], x)
    for i in (9, 10, 11):
        x = residual_bottleneck(t[i], x)
    x = gdn(t[13], residual_block_with_stride(t[12], x))
    x = conv(t[15], x, pad=(1, 1, 2, 2))
    return win_noshift_attention(t[16], x)


def synthesis(m, x):
    """synthesisTransformModel (net_ga.py:364-403)."""
    t = m.transform
    x = win_noshift_attention(t[0], x)
    x = gdn(t[3], conv_t(t[2], x))
    x = gdn(t[6], conv_t(t[5], x))
    x = win_noshift_attention(t[7], x)
    x = gdn(t[10], conv_t(t[9], x))
    return gdn(t[13], conv_t(t[12], x))


def seq_gelu(seq, x):
    """conv (GELU conv)* hyper stacks (net_ga.py:811-845); subpel = conv3x3 + PixelShuffle(2)."""
    mods = [m for m in seq if not isinstance(m, nn.GELU)]
    for k, m in enumerate(mods):
        act = ACT_NONE if k == len(mods) - 1 else ACT_GELU
        if isinstance(m, nn.Sequential):
            x = pixel_shuffle(conv(m[0], x, act))   # GELU commutes with the shuffle
        else:
            x = conv(m, x, act)
    return x


def syntax(m, s):
    """Syntax_Model (net_ga.py:626-647) + bypass_round (:1016, straight-through)."""
    ds = lambda d, x: conv(d.pointwise, conv(d.depthwise, x))
    p1 = AG.avgpool(s)
    ds1 = conv(m.down0, ds(m.Depth_down0, s), ACT_RELU)
    p2 = AG.avgpool(ds1)
    ds2 = conv(m.down1, ds(m.Depth_down1, ds1), ACT_RELU)
    ds2 = win_noshift_attention(m.WAM, ds2)
    p3 = AG.avgpool(ds2)
    ds3 = conv(m.down2, ds(m.Depth_down2, ds2), ACT_RELU)
    p4 = AG.avgpool(ds3)
    return conv(m.conv, torch.cat([p1, p2, p3, p4], -1), ACT_ROUND)


def generator(m, s):
    """conv_generator (net_ga.py:597-604): [B,1,1,M] -> [B,1,1,3*M] (row-major (3, M))."""
    t = m.transform
    h = linear(t[0], s, ACT_LRELU, 0.2)
    h = linear(t[2], h, ACT_LRELU, 0.2)
    return linear(t[4], h)


# --------------------------------------------------------------------------- net_unet_ha_hs hyper nets
def _c(x):
    return x.contiguous()


def residual_block3_5(m, x):
    """ResidualBlock3_5 (Block_unet.py:295-332): lrelu(conv3x3) lrelu(conv5x5) lrelu(conv3x3) + x."""
    t = conv(m.conv1, x, ACT_LRELU)
    t = conv(m.conv2, t, ACT_LRELU)
    idn = conv(m.skip, x) if m.skip is not None else x
    return AG.add(conv(m.conv3, t, ACT_LRELU), idn)


def residual_block5x5(m, x):
    """ResidualBlock5x5 (Block_unet.py:335-364): lrelu(conv5x5(x)) + x."""
    idn = conv(m.skip, x) if m.skip is not None else x
    return AG.add(conv(m.conv2, x, ACT_LRELU), idn)


def residual_block3x3(m, x):
    """ResidualBlock3x3 (Block_unet.py:367-398): lrelu(conv3x3) lrelu(conv3x3) + x."""
    t = conv(m.conv1, x, ACT_LRELU)
    idn = conv(m.skip, x) if m.skip is not None else x
    return AG.add(conv(m.conv3, t, ACT_LRELU), idn)


def conv_t1(m, x, act: int = ACT_NONE):
    """nn.ConvTranspose2d without the ZeroPad2d pre-pad (Block_unet.py up1..up4)."""
    return AG.conv_transpose2d(x, m.weight, m.bias, m.stride[0], m.padding[0], m.output_padding[0], (0, 0), act)


def unet_ha_new(m, x):
    """Unet_ha_new.forward (Block_unet.py:815-838) -> (z, middle_x, down_x1, x)."""
    C = x.shape[-1]
    h = C // 2
    cat1 = torch.cat([residual_block3_5(m.conv1, _c(x[..., h:])), wba(m.SpatialTransformer1, _c(x[..., :h]))], -1)
    d = conv(m.down0, cat1, residual=x)
    down_x1 = conv(m.down1, d, ACT_GELU)
    cat2 = torch.cat([residual_block5x5(m.conv2, _c(down_x1[..., :128])),
                      wba(m.SpatialTransformer2, _c(down_x1[..., 128:]))], -1)
    d2 = conv(m.down2, conv(m.down3, cat2, residual=down_x1), ACT_GELU)
    mm = residual_bottleneck(m.middle[0], d2)
    mm = wba(m.middle[1], mm)
    mm = residual_bottleneck(m.middle[2], mm)
    return mm, mm, down_x1, x


def unet_hs_new(m, middle_x, down_x1, inp):
    """Unet_hs_new.forward (Block_unet.py:868-890); its first argument (z_hat) is never read."""
    cat0 = torch.cat([residual_block3x3(m.conv3, _c(middle_x[..., 256:])),
                      wba(m.SpatialTransformer3, _c(middle_x[..., :256]))], -1)
    u = conv(m.up0, cat0, residual=middle_x)
    u1 = conv_t1(m.up3, torch.cat([conv_t1(m.up1, u, ACT_GELU), down_x1], -1), ACT_GELU)
    cat2 = torch.cat([residual_block3x3(m.conv4, _c(u1[..., :128])), wba(m.SpatialTransformer2, _c(u1[..., 128:]))],
                     -1)
    u2 = conv(m.up5, cat2, residual=u1)
    u2 = conv_t1(m.up2, u2, ACT_GELU)
    return conv_t1(m.up4, torch.cat([u2, inp], -1))


# --------------------------------------------------------------------------- Net
def _cc(seq, x):
    """cc_mean / cc_scale / lrp transforms: conv3x3 GELU conv3x3 GELU conv3x3."""
    return conv(seq[4], conv(seq[2], conv(seq[0], x, ACT_GELU), ACT_GELU))


def net_forward_train(net, inputs: torch.Tensor, seed: int, seed_dev=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """net_ga.Net.forward(inputs, 'train') -> (bpp, mse), differentiable through liblic
    (net_unet_ha_hs.Net: the U-Net hyper nets of net_unet_ha_hs.py:880-895)."""
    if net.arch not in ("net_ga", "net_unet_ha_hs"):
        raise NotImplementedError(f"train mode is not implemented for {net.arch}")
    if net.post_processing:
        raise NotImplementedError("train mode with post_processing (HAN) is not implemented")
    if not inputs.is_cuda:
        raise RuntimeError("lic_amd Net runs on the GPU only (HIP path); move inputs to cuda")
    x_in = inputs.contiguous().float()
    B, _, H, W = x_in.shape
    if H % 64 or W % 64:
        raise ValueError("Net.forward: H and W must be multiples of 64")
    _, h, w, _ = net.train_size
    dev, dt = x_in.device, net.dtype
    x = AG.to_nhwc(x_in, dt)
    z3 = analysis(net.a_model, x)                                     # :988
    if net.arch == "net_ga":
        z = seq_gelu(net.h_a, z3)                                     # :993
        z_hat = AG.ste_quantize(z, net._medians(dev))                 # :996-1003
        latent_scales = seq_gelu(net.h_scale_s, z_hat)                # :1006
        latent_means = seq_gelu(net.h_mean_s, z_hat)                  # :1007
    else:
        # net_unet_ha_hs.py:880-895: h_s reads encoder-side features, not z_hat, and the two
        # identical h_s calls give latent_scales == latent_means (one call, its gradient sums
        # both uses exactly as the reference's two calls do)
        z, middle_x, down_x1, inp = unet_ha_new(net.h_a, z3)
        latent_scales = latent_means = unet_hs_new(net.h_s, middle_x, down_x1, inp)
    syn = syntax(net.syntax_model, z3[..., :net.M].contiguous())      # :1013-1016
    cw = generator(net.conv_weights_gen, syn)                         # :1083
    sw = 192 // net.num_slices
    num_pixels = B * h * w
    gc = net.gaussian_conditional
    y_hats = []
    bpp = None
    for i in range(net.num_slices):                                   # :1025-1067
        support = y_hats[:net.max_support_slices]
        ms = swatten(net.atten_mean[i][0], torch.cat([latent_means] + support, -1))
        mu = _cc(net.cc_mean_transforms[i], ms)
        ss = swatten(net.atten_scale[i][0], torch.cat([latent_scales] + support, -1))
        sc = _cc(net.cc_scale_transforms[i], ss)
        y_i = z3[..., sw * i:sw * (i + 1)].contiguous()
        if seed_dev is None:
            b_i, yq = AG.rate_train(y_i, mu, sc, seed * net.num_slices + i, num_pixels, gc._scale_bound,
                                    gc._likelihood_bound)
        else:   # captured step: the kernels read the step's seed from the device
            b_i, yq = AG.rate_train(y_i, mu, sc, i, num_pixels, gc._scale_bound, gc._likelihood_bound,
                                    seed_dev=seed_dev, seed_mul=net.num_slices)
        bpp = b_i if bpp is None else bpp + b_i
        lrp = _cc(net.lrp_transforms[i], torch.cat([ms, yq], -1))
        y_hats.append(AG.half_tanh_add(lrp, yq))                      # y_hat + 0.5 tanh(lrp)
    y_hat = torch.cat(y_hats, -1)
    x16 = synthesis(net.s_model, y_hat)                               # :1078
    mse = AG.recon_mse(x16, cw, x_in)                                 # :1089-1092, :1115
    return bpp, mse
