"""Training path: forward + backward of the liblic autograd
layers (lic_amd.autograd) against plain fp32 PyTorch CPU autograd of the same op on
the same seeded inputs and upstream gradients.

Tolerances: fp32 path — relative 1e-4 of each gradient's max magnitude (the MFMA
wgrad sums ~1e3-1e5 products per element in a different order than oneDNN);
fp16 path — 2e-2 of the max magnitude (fp16 operands, fp32 accumulation)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
DTYPES = [torch.float32, torch.float16]


def _rel(out, ref, dtype, name):
    out = out.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert out.shape == ref.shape, (name, out.shape, ref.shape)
    scale = ref.abs().max().item() + 1e-12
    err = (out - ref).abs().max().item()
    tol = 2e-2 if dtype == torch.float16 else 1e-4
    assert err <= tol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e} ({dtype})"


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _run(fn_gpu, fn_ref, x, params, dtype, seed=3):
    """Compare forward outputs and grads of x and params; upstream grad seeded."""
    g = torch.Generator().manual_seed(seed)
    xr = x.clone().requires_grad_(True)
    pr = [p.clone().requires_grad_(True) for p in params]
    yr = fn_ref(xr, *pr)
    dy = torch.randn(yr.shape, generator=g)
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
