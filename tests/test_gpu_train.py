"""Training path: forward + backward of the liblic autograd
layers (lic_amd.autograd) against plain fp32 PyTorch CPU autograd of the same op on
the same seeded inputs and upstream gradients.

Tolerances: fp32 path — relative 1e-4 of each gradient's max magnitude (the MFMA
wgrad sums ~1e3-1e5 products per element in a different order than oneDNN);
fp16 path — 2e-2 of the max magnitude (fp16 operands, fp32 accumulation)."""
import contextlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
DTYPES = [torch.float32, torch.float16, torch.bfloat16]
TOL16 = {torch.float16: 2e-2, torch.bfloat16: 4e-2}   # of the tensor scale; fp32: 1e-4


def _rel(out, ref, dtype, name):
    out = out.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert out.shape == ref.shape, (name, out.shape, ref.shape)
    scale = ref.abs().max().item() + 1e-12
    err = (out - ref).abs().max().item()
    if dtype == torch.bfloat16:
        # 8 mantissa bits: a pre-activation within ~1e-2 of a ReLU / LeakyReLU kink can take the
        # other branch than in fp32, so single entries of dx may differ by |dz|; bar on the norm
        rel = ((out - ref).norm() / (ref.norm() + 1e-12)).item()
        assert rel <= 3e-2 and err <= 0.2 * scale, f"{name}: rel norm err {rel:.3e}, max {err:.3e} vs {scale:.3e}"
        return
    tol = TOL16.get(dtype, 1e-4)
    assert err <= tol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e} ({dtype})"


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _run(fn_gpu, fn_ref, x, params, dtype, seed=3):
    """Compare forward outputs and grads of x and params; upstream grad seeded."""
    g = torch.Generator().manual_seed(seed)
    if dtype != torch.float32:   # the reference sees the same 16-bit-rounded activations and
        x = x.to(dtype).float()  # packed weights (biases stay fp32 in the kernels)
        params = [p.to(dtype).float() if p.dim() >= 2 else p for p in params]
    xr = x.clone().requires_grad_(True)
    pr = [p.clone().requires_grad_(True) for p in params]
    yr = fn_ref(xr, *pr)
    dy = torch.randn(yr.shape, generator=g)
    if dtype != torch.float32:
        dy = dy.to(dtype).float()
    yr.backward(dy)

    xg = _nhwc(x).to(DEV, dtype).requires_grad_(True)
    pg = [p.to(DEV).requires_grad_(True) for p in params]
    yg = fn_gpu(xg, *pg)
    yg.backward(_nhwc(dy).to(DEV, dtype))
    torch.cuda.synchronize()
    _rel(_nchw(yg), yr, dtype, "y")
    _rel(_nchw(xg.grad), xr.grad, dtype, "dx")
    for i, (a, b) in enumerate(zip(pg, pr)):
        _rel(a.grad, b.grad, dtype, f"dparam{i}")


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("act,res_act", [("none", False), ("relu", True), ("lrelu", True), ("gelu", True)])
def test_conv2d_residual_grad(dtype, act, res_act):
    """conv2d(..., residual=r): conv + r in the conv epilogue (residual_bottleneck, the proj / MLP
    Linears, the U-Net skips), res_act: act(conv + r) (compressai ResidualUnit's relu(conv + x)); the
    residual's gradient is the conv output's."""
    from lic_amd import autograd as AG
    from lic_amd._ffi import ACT_GELU, ACT_LRELU, ACT_NONE, ACT_RELU
    code = {"none": ACT_NONE, "gelu": ACT_GELU, "lrelu": ACT_LRELU, "relu": ACT_RELU}[act]
    ref_act = {"none": lambda v: v, "gelu": F.gelu, "lrelu": lambda v: F.leaky_relu(v, 0.01), "relu": F.relu}[act]
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 32, 12, 12, generator=g)
    w = torch.randn(48, 32, 3, 3, generator=g) / (32 * 9) ** 0.5
    b = torch.randn(48, generator=g) * 0.1
    r = torch.randn(2, 48, 12, 12, generator=g)
    _run(lambda xg, wg, bg, rg: AG.conv2d(xg, wg, bg, 1, 1, code, residual=_nhwc(rg).to(xg.dtype), res_act=res_act),
         lambda xr, wr, br, rr: ref_act(F.conv2d(xr, wr, br, 1, 1) + rr), x, [w, b, r], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("ci,co,k,s,pad", [
    (64, 64, 3, 1, 1),     # RB / WNSA conv3x3
    (192, 192, 3, 1, 1),   # full-width 3x3 (128-wide wgrad tiles)
    (32, 96, 1, 1, 0),     # 1x1
    (64, 32, 7, 1, 3),     # conv7x7 of conv_b
    (32, 64, 3, 2, 1),     # RBWS conv3x3 s2
    (3, 64, 3, 2, 1),      # image layer (3 channels padded to 16 B)
    (64, 3, 3, 1, 1),      # 3-channel output (dz padded)
])
def test_conv2d_grad(dtype, ci, co, k, s, pad):
    from lic_amd import autograd as AG
    from lic_amd._ffi import ACT_NONE
    g = torch.Generator().manual_seed(ci * 7 + co + k)
    x = torch.randn(2, ci, 20, 24, generator=g)
    w = torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5
    b = torch.randn(co, generator=g) * 0.1
    _run(lambda xg, wg, bg: AG.conv2d(xg, wg, bg, s, pad, ACT_NONE),
         lambda xr, wr, br: F.conv2d(xr, wr, br, s, pad), x, [w, b], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv5x5_s2_zeropad_grad(dtype):
    """ZeroPad2d((1,2,1,2)) + Conv2d(k5, s2, p0) (net_ga.py:277-282)."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 32, 16, 16, generator=g)
    w = torch.randn(64, 32, 5, 5, generator=g) / (32 * 25) ** 0.5
    b = torch.randn(64, generator=g) * 0.1
    _run(lambda xg, wg, bg: AG.conv2d(xg, wg, bg, 2, (1, 1, 2, 2)),
         lambda xr, wr, br: F.conv2d(F.pad(xr, (1, 2, 1, 2)), wr, br, 2), x, [w, b], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("act", ["gelu", "lrelu", "relu"])
def test_conv2d_act_grad(dtype, act):
    from lic_amd import autograd as AG
    from lic_amd._ffi import ACT_GELU, ACT_LRELU, ACT_RELU
    code = {"gelu": ACT_GELU, "lrelu": ACT_LRELU, "relu": ACT_RELU}[act]
    ref_act = {"gelu": F.gelu, "lrelu": lambda v: F.leaky_relu(v, 0.01), "relu": F.relu}[act]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 32, 12, 12, generator=g)
    w = torch.randn(32, 32, 3, 3, generator=g) / (32 * 9) ** 0.5
    b = torch.randn(32, generator=g) * 0.1
    _run(lambda xg, wg, bg: AG.conv2d(xg, wg, bg, 1, 1, code),
         lambda xr, wr, br: ref_act(F.conv2d(xr, wr, br, 1, 1)), x, [w, b], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("ci,co,prepad", [(64, 64, (1, 1)), (64, 16, (1, 1)), (32, 48, (0, 0))])
def test_conv_transpose_k5s2_grad(dtype, ci, co, prepad):
    """ZeroPad2d((1,0,1,0)) + ConvTranspose2d(k5, s2, p3, op1) (net_ga.py:373-397)."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(ci + co)
    x = torch.randn(2, ci, 8, 10, generator=g)
    w = torch.randn(ci, co, 5, 5, generator=g) / (ci * 6.25) ** 0.5
    b = torch.randn(co, generator=g) * 0.1
    p, op = (3, 1) if prepad != (0, 0) else (2, 1)

    def ref(xr, wr, br):
        if prepad != (0, 0):
            xr = F.pad(xr, (prepad[1], 0, prepad[0], 0))
        return F.conv_transpose2d(xr, wr, br, 2, p, op)

    _run(lambda xg, wg, bg: AG.conv_transpose2d(xg, wg, bg, 2, p, op, prepad), ref, x, [w, b], dtype)


def _gdn_ref(x, beta, gamma, bb, gb, ped, inverse):
    from oracle import ref_cpu as R  # noqa: F401  (oracle defines the forward; autograd via LowerBound rule)

    class LB(torch.autograd.Function):
        @staticmethod
        def forward(ctx, v, bound):
            ctx.save_for_backward(v)
            ctx.bound = bound
            return torch.clamp(v, min=bound)

        @staticmethod
        def backward(ctx, go):
            (v,) = ctx.saved_tensors
            return ((v >= ctx.bound) | (go < 0)).to(go.dtype) * go, None

    be = LB.apply(beta, bb) ** 2 - ped
    ga = LB.apply(gamma, gb) ** 2 - ped
    C = x.shape[1]
    n = F.conv2d(x * x, ga.view(C, C, 1, 1), be)
    return x * torch.sqrt(n) if inverse else x / torch.sqrt(n)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("C", [64, 192])
def test_gdn_grad(dtype, inverse, C):
    """model/gdn.py GDN / IGDN incl. the LowerBound gradient rule (model/gdn.py:18-26)."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(C + inverse)
    ped = (2 ** -18) ** 2
    bb, gb = (1e-6 + ped) ** 0.5, 2 ** -18
    x = torch.randn(2, C, 10, 12, generator=g)
    beta = torch.sqrt(torch.ones(C) + ped) + 0.05 * torch.randn(C, generator=g)
    gamma = torch.sqrt(0.1 * torch.eye(C) + ped) + 0.01 * torch.rand(C, C, generator=g)
    gamma[0, 1] = 0.0  # below the bound: exercises the LowerBound pass-through rule
    _run(lambda xg, b_, g_: AG.gdn(xg, b_, g_, bb, gb, ped, inverse),
         lambda xr, b_, g_: _gdn_ref(xr, b_, g_, bb, gb, ped, inverse), x, [beta, gamma], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_channel_sum(dtype):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 17, 19, 40, generator=g)
    out = AG.channel_sum(x.to(DEV, dtype))
    ref = x.to(dtype).float().sum(dim=(0, 1, 2))
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32])
def test_wgrad_large_k(dtype):
    """B*H*W = 32*64*64 output pixels (the 64x64 WNSA conv of a 256x256 batch of 32): split-K
    partials + reduce over the full size."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(9)
    x = torch.randn(32, 64, 64, 64, generator=g)
    dz = torch.randn(32, 64, 64, 64, generator=g)
    dw = torch.empty((64, 64, 3, 3), dtype=torch.float32, device=DEV)
    tdy, tdx = AG._taps(3, 3, 1, 1)
    AG.wgrad(x.to(DEV), dz.to(DEV), tdy, tdx, dw=dw, strides=(64 * 9, 9, 1), co_out=64, ci_out=64)
    ref = torch.nn.grad.conv2d_weight(_nchw(x), (64, 64, 3, 3), _nchw(dz), padding=1)
    _rel(dw, ref, dtype, "dw")


# --------------------------------------------------------------------------- ops of the full training graph
class _LBFn(torch.autograd.Function):
    """ops/bound_ops.py:25-28 LowerBound gradient rule (pass if x >= bound or grad < 0)."""

    @staticmethod
    def forward(ctx, v, bound):
        ctx.save_for_backward(v)
        ctx.bound = bound
        return torch.clamp(v, min=bound)

    @staticmethod
    def backward(ctx, go):
        (v,) = ctx.saved_tensors
        return ((v >= ctx.bound) | (go < 0)).to(go.dtype) * go, None


def _check(gpu_fn, ref_fn, tensors, act, dtype, seed=0):
    """Forward outputs and input grads of gpu_fn vs the fp32 CPU autograd of ref_fn; tensors are CPU
    fp32, act[i] says whether input i is an activation (cast to dtype) or an fp32 parameter."""
    g = torch.Generator().manual_seed(seed)
    rs = [t.clone().requires_grad_(True) for t in tensors]
    outs_r = ref_fn(*rs)
    outs_r = outs_r if isinstance(outs_r, tuple) else (outs_r,)
    gs = [torch.randn(o.shape, generator=g) for o in outs_r]
    torch.autograd.backward(outs_r, gs)
    gt = [t.to(DEV, dtype if a else torch.float32).requires_grad_(True) for t, a in zip(tensors, act)]
    outs_g = gpu_fn(*gt)
    outs_g = outs_g if isinstance(outs_g, tuple) else (outs_g,)
    torch.autograd.backward(outs_g, [gg.to(DEV, o.dtype) for gg, o in zip(gs, outs_g)])
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(zip(outs_g, outs_r)):
        _rel(o, r, dtype, f"out{i}")
    for i, (a_, r) in enumerate(zip(gt, rs)):
        if r.grad is not None:
            _rel(a_.grad, r.grad, dtype, f"grad{i}")


def _attn_core_ref(qkv, table, C, heads, ws, shift, wmsa):
    """WBA (layers/win_attention.py:85-116, 154-209) / WMSA (model/Block_unet.py:216-252) attention
    core from a qkv map, written with the oracle's window helpers."""
    from oracle import ref_cpu as R
    B, H, W, _ = qkv.shape
    d, N = C // heads, ws * ws
    x = torch.roll(qkv, (-shift, -shift), (1, 2)) if shift else qkv
    t = R.window_partition(x, ws).view(-1, N, 3, heads, d).permute(2, 0, 3, 1, 4)
    q, k, v = t[0], t[1], t[2]
    scale = d ** -0.5
    attn = (q @ k.transpose(-2, -1)) * scale if wmsa else (q * scale) @ k.transpose(-2, -1)
    rpi = R.relative_position_index(ws).view(-1)
    rpb = table.reshape(heads, -1)[:, rpi].view(heads, N, N) if wmsa else table[rpi].view(N, N, heads).permute(2, 0, 1)
    attn = attn + rpb.unsqueeze(0)
    nW = (H // ws) * (W // ws)
    if shift and not wmsa:
        attn = (attn.view(B, nW, heads, N, N) + R.wba_mask(H, W, ws, shift).unsqueeze(1).unsqueeze(0)).view(-1, heads, N, N)
    if shift and wmsa:
        m = R.wmsa_mask(H // ws, W // ws, ws, shift)
        attn = attn.view(B, nW, heads, N, N).masked_fill(m.unsqueeze(0).unsqueeze(2), float("-inf")).view(-1, heads, N, N)
    o = (torch.softmax(attn, -1) @ v).transpose(1, 2).reshape(-1, ws, ws, C)
    o = R.window_reverse(o, ws, H, W)
    return torch.roll(o, (shift, shift), (1, 2)) if shift else o


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("ws,shift,wmsa,C", [(8, 4, False, 192), (8, 0, False, 64), (4, 2, False, 64), (8, 2, False, 256),
                                             (2, 1, False, 64), (8, 4, True, 128), (8, 0, True, 128)])
def test_win_attn_grad(dtype, ws, shift, wmsa, C):
    from lic_amd import autograd as AG
    heads = 8
    g = torch.Generator().manual_seed(ws * 10 + shift + C)
    qkv = torch.randn(2, 16, 16, 3 * C, generator=g)
    R_ = (2 * ws - 1) ** 2
    table = (torch.randn(heads, 2 * ws - 1, 2 * ws - 1, generator=g) if wmsa else torch.randn(R_, heads, generator=g))
    table = table * 0.5
    _check(lambda x, t: AG.win_attn(x, t, C, heads, ws, shift, tab_sr=1 if wmsa else heads, tab_sh=R_ if wmsa else 1,
                                    mask_kind=(2 if wmsa else 1) if shift else 0, scale_after=wmsa,
                                    scale=(C // heads) ** -0.5),
           lambda x, t: _attn_core_ref(x, t, C, heads, ws, shift, wmsa), [qkv, table], [True, False], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("C", [128, 192])
def test_layernorm_grad(dtype, C):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(C)
    x = torch.randn(2, 8, 8, C, generator=g) * 2 + 0.5
    w = 1 + 0.1 * torch.randn(C, generator=g)
    b = 0.1 * torch.randn(C, generator=g)
    _check(lambda x_, w_, b_: AG.layernorm(x_, w_, b_, 1e-5), lambda x_, w_, b_: F.layer_norm(x_, (C,), w_, b_, 1e-5),
           [x, w, b], [True, False, False], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_elementwise_grads(dtype):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(1)
    a, b, r = (torch.randn(2, 6, 7, 48, generator=g) for _ in range(3))
    _check(AG.gate, lambda b_, a_, r_: a_ * torch.sigmoid(b_) + r_, [b, a, r], [True] * 3, dtype)
    _check(AG.half_tanh_add, lambda x_, r_: r_ + 0.5 * torch.tanh(x_), [a, r], [True] * 2, dtype)
    _check(AG.add, lambda x_, y_: x_ + y_, [a, b], [True] * 2, dtype)
    _check(AG.avgpool, lambda x_: x_.mean((1, 2), keepdim=True), [a], [True], dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_dwconv_grad(dtype):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(2)
    C = 32
    x = torch.randn(2, 16, 16, C, generator=g)
    w = torch.randn(C, 1, 3, 3, generator=g) / 3
    b = 0.1 * torch.randn(C, generator=g)
    _check(lambda x_, w_, b_: AG.dwconv2d(x_, w_, b_, 1, 1),
           lambda x_, w_, b_: F.conv2d(x_.permute(0, 3, 1, 2), w_, b_, 1, 1, 1, C).permute(0, 2, 3, 1),
           [x, w, b], [True, False, False], dtype)


def _noise_ref(seed, n):
    """The rate kernels' counter-based U(-1/2, 1/2) noise (train.hip noise_u), restated in numpy."""
    import numpy as np
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        z = np.array([seed], dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + i
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0) - np.float32(0.5)
    return torch.from_numpy(u)


def _rate_ref(y, mu, sc, seed, num_pixels):
    """compressai GaussianConditional.forward in training mode (noise) + LowerBound rules, and
    ste_round(y - mu) + mu (net_ga.py:1049-1053); y, mu, sc NHWC."""
    import math
    u = _noise_ref(seed, y.numel()).view(y.shape)
    v = ((y + u) - mu).abs()
    s = _LBFn.apply(sc, 0.11)
    c = -(2 ** -0.5)
    L = 0.5 * torch.erfc(c * ((0.5 - v) / s)) - 0.5 * torch.erfc(c * ((-0.5 - v) / s))
    L = _LBFn.apply(L, 1e-9)
    bpp = torch.log(L).sum() / (-math.log(2) * num_pixels)
    d = y - mu
    return bpp, (torch.round(d) - d.detach() + d) + mu


@pytest.mark.parametrize("dtype", DTYPES)
def test_rate_train_grad(dtype):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(5)
    y = torch.randn(2, 8, 8, 48, generator=g) * 3
    mu = torch.randn(2, 8, 8, 48, generator=g)
    sc = torch.rand(2, 8, 8, 48, generator=g) * 2 - 0.2     # some scales under the 0.11 bound
    if dtype != torch.float32:   # the reference sees the same 16-bit-rounded inputs
        y, mu, sc = y.to(dtype).float(), mu.to(dtype).float(), sc.to(dtype).float()
    _check(lambda a, b, c: AG.rate_train(a, b, c, 77, 2 * 128 * 128),
           lambda a, b, c: _rate_ref(a, b, c, 77, 2 * 128 * 128), [y, mu, sc], [True] * 3, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_recon_mse_grad(dtype):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(6)
    x16 = torch.randn(2, 32, 32, 16, generator=g) * 0.5
    cw = torch.randn(2, 1, 1, 48, generator=g) * 0.3
    img = torch.rand(2, 3, 32, 32, generator=g) * 2 - 1

    def ref(x_, w_):
        xt = torch.tanh(torch.einsum("bhwc,boc->bohw", x_, w_.view(2, 3, 16)))
        return ((xt - img) ** 2).mean()

    _check(lambda x_, w_: AG.recon_mse(x_, w_, img.to(DEV)), ref, [x16, cw], [True, True], dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_wgrad_defer_bit_identical(dtype):
    """autograd.WgradDefer (the split-K wgrad reduces of a backward as one lic_wgrad_reduce_batch
    launch after it) gives the same dw / db / dx bits as the per-layer reduce: a 3x3 (bias, GELU),
    a 1x1, a stride-2 3x3, a 5x5 s2 ZeroPad conv and a transposed conv, eagerly and replayed from a
    hipGraph capture (the table filled by finalize())."""
    from lic_amd import autograd as AG
    from lic_amd._ffi import ACT_GELU
    torch.manual_seed(5)
    x0 = torch.randn(2, 32, 32, 64, device=DEV).to(dtype)
    ws = [torch.randn(64, 64, 3, 3, device=DEV) * 0.05, torch.randn(96, 64, 1, 1, device=DEV) * 0.1,
          torch.randn(64, 96, 3, 3, device=DEV) * 0.05, torch.randn(64, 64, 5, 5, device=DEV) * 0.03,
          torch.randn(64, 32, 5, 5, device=DEV) * 0.03]
    bs = [torch.randn(w.shape[0] if i != 4 else 32, device=DEV) * 0.1 for i, w in enumerate(ws)]
    dy = torch.randn(2, 16, 16, 32, device=DEV).to(dtype)

    def step(defer):
        x = x0.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(True) for t in ws + bs]
        w, b = ps[:5], ps[5:]
        h = AG.conv2d(x, w[0], b[0], 1, 1, ACT_GELU)
        h = AG.conv2d(h, w[1], b[1], 1, 0)
        h = AG.conv2d(h, w[2], b[2], 2, 1)
        h = AG.conv2d(h, w[3], b[3], 1, (1, 1, 2, 2))[:, :8, :8].contiguous()
        y = AG.conv_transpose2d(h, w[4], b[4], 2, 3, 1, (1, 1))
        with defer if defer is not None else contextlib.nullcontext():
            y.backward(dy[:, :y.shape[1], :y.shape[2]].contiguous())
        return [x.grad] + [p.grad for p in ps]

    ref = step(None)
    d = AG.WgradDefer()
    got = step(d)
    torch.cuda.synchronize()
    for i, (r, g) in enumerate(zip(ref, got)):
        assert torch.equal(r, g), f"gradient {i} differs with the deferred reduce"
    # captured: the table is sized by the eager run above, filled after the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        step(d)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            outs = step(d)
    d.finalize()
    graph.replay()
    torch.cuda.synchronize()
    for i, (r, g) in enumerate(zip(ref, outs)):
        assert torch.equal(r, g), f"gradient {i} differs in the captured deferred step"
