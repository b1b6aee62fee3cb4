"""Weight gradient of the 16-bit training path (lic_conv2d_wgrad -> wgrad_tr_kernel for 1x1, 3x3,
5x5 and 7x7 tap windows, wgrad_kernel otherwise) against float64 torch on the SAME 16-bit operands.

Both sides see identical bf16 / fp16 inputs, so the only difference is the fp32 MFMA
accumulation order: the bar is 2e-5 of the gradient's max magnitude (an indexing error — a
wrong tap, pixel or channel — is O(1) of it).  Covers ragged lattices (maps not multiples of
the 8x8 tile), channel counts that are not multiples of the 64-wide blocks, stride 2 with the
asymmetric ZeroPad of net_ga.py:277-282, the transposed-conv wgrad (roles of x and dz exchanged
on an (H, W) lattice), the GDN x^2 prologue and a split-K size of config 5's batch."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _check(dw, ref, name):
    ref = ref.double()
    scale = ref.abs().max().item() + 1e-30
    err = (dw.double().cpu() - ref).abs().max().item()
    assert err <= 2e-5 * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


SHAPES = [
    (2, 20, 24, 64, 64, 3, 1, (1, 1, 1, 1)),       # ragged 8x8 tiles
    (1, 16, 16, 192, 128, 3, 1, (1, 1, 1, 1)),     # 3 x 2 channel blocks
    (2, 12, 10, 96, 40, 3, 1, (1, 1, 1, 1)),       # partial 64-wide blocks on both sides
    (2, 18, 14, 32, 96, 1, 1, (0, 0, 0, 0)),       # 1x1 (16 x 8 tiles)
    (2, 18, 14, 128, 64, 1, 1, (0, 0, 0, 0)),      # 1x1, two ci blocks as virtual taps
    (1, 20, 12, 320, 96, 1, 1, (0, 0, 0, 0)),      # 1x1, 5 ci blocks -> 4 + 1 (partial group)
    (1, 16, 16, 256, 192, 1, 1, (0, 0, 0, 0)),     # 1x1, 4 virtual taps
    (2, 16, 16, 32, 64, 5, 2, (1, 1, 2, 2)),       # ZeroPad2d((1, 2, 1, 2)) + conv5x5 s2
    (2, 17, 15, 64, 64, 3, 2, (1, 1, 1, 1)),       # conv3x3 s2, odd map
    (1, 12, 12, 64, 32, 5, 1, (2, 2, 2, 2)),       # 5x5 s1 (rows of 5 taps)
    (1, 12, 12, 32, 64, 7, 1, (3, 3, 3, 3)),       # 7x7 (rows of 7 taps)
    (1, 10, 10, 32, 64, 7, 2, (3, 3, 3, 3)),       # 7x7 s2
    (1, 11, 13, 32, 48, 2, 1, (0, 0, 1, 1)),       # 2x2: the generic kernel
    (1, 9, 9, 16, 64, 1, 2, (0, 0, 0, 0)),         # 1x1 s2
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,W,ci,co,k,s,pad", SHAPES)
def test_conv_wgrad(dtype, B, H, W, ci, co, k, s, pad):
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(B * 1000 + H * 31 + ci + co + k + s)
    pt, pl, pb, pr = pad
    Ho = (H + pt + pb - k) // s + 1
    Wo = (W + pl + pr - k) // s + 1
    x = torch.randn(B, H, W, ci, generator=g).to(dtype)
    dz = torch.randn(B, Ho, Wo, co, generator=g).to(dtype)
    dw = torch.empty((co, ci, k, k), dtype=torch.float32, device=DEV)
    tdy, tdx = AG._taps(k, k, pt, pl)
    AG.wgrad(x.to(DEV), dz.to(DEV), tdy, tdx, stride=s, dw=dw, strides=(ci * k * k, k * k, 1), co_out=co,
             ci_out=ci)
    torch.cuda.synchronize()
    xp = torch.nn.functional.pad(_nchw(x).double(), (pl, pr, pt, pb))
    ref = torch.nn.grad.conv2d_weight(xp, (co, ci, k, k), _nchw(dz).double(), stride=s)
    _check(dw, ref, f"wgrad k{k} s{s}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_convT_wgrad(dtype):
    """ConvTranspose2d k5 s2 p2 op1 (prepad (1, 1)) weight gradient as autograd.py's _ConvT2dFn
    computes it: dW[c, n] = sum_i x[i, c] * dz[s*i + tap, n] over the input lattice."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(5)
    B, H, W, ci, co = 2, 9, 11, 64, 48
    x = torch.randn(B, ci, H, W, generator=g).to(dtype)
    w = torch.randn(ci, co, 5, 5, generator=g)
    xr = x.double().requires_grad_(False)
    wr = w.double().requires_grad_(True)
    y = torch.nn.functional.conv_transpose2d(xr, wr, stride=2, padding=2, output_padding=1)
    dy = torch.randn(y.shape, generator=g).to(dtype)
    y.backward(dy.double())
    s, p, prepad = 2, 2, (0, 0)
    pt, pl = p - s * prepad[0], p - s * prepad[1]
    dw = torch.empty((ci, co, 5, 5), dtype=torch.float32, device=DEV)
    tdy, tdx = AG._taps(5, 5, pt, pl)
    dzn = dy.permute(0, 2, 3, 1).contiguous().to(DEV)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    AG.wgrad(dzn, xn, tdy, tdx, stride=s, lattice=(H, W), dw=dw, strides=(co * 25, 25, 1), co_out=ci, ci_out=co)
    torch.cuda.synchronize()
    _check(dw, wr.grad, "convT wgrad")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gdn_square_wgrad(dtype):
    """dGamma' = sum_pix u[pix, n] * x[pix, c]^2 (PRO_SQUARE; x^2 rounded to the 16-bit type as
    the forward's conv operand is)."""
    from lic_amd import autograd as AG
    from lic_amd._ffi import PRO_SQUARE
    g = torch.Generator().manual_seed(7)
    B, H, W, C = 2, 13, 19, 192
    x = torch.randn(B, H, W, C, generator=g).to(dtype)
    u = torch.randn(B, H, W, C, generator=g).to(dtype)
    dw = torch.empty((C, C), dtype=torch.float32, device=DEV)
    AG.wgrad(x.to(DEV), u.to(DEV), [0], [0], dw=dw, strides=(C, 1, 0), co_out=C, ci_out=C, prologue=PRO_SQUARE)
    torch.cuda.synchronize()
    x2 = (x.float() * x.float()).to(dtype).double().reshape(-1, C)
    ref = u.double().reshape(-1, C).t() @ x2
    _check(dw, ref, "gdn wgrad")


@pytest.mark.parametrize("dtype", [torch.bfloat16])
@pytest.mark.parametrize("C,HW", [(128, 128), (192, 32)])
def test_wgrad_config5_split_k(dtype, C, HW):
    """Config 5 sizes (batch 8): 3x3 at 128^2 (2048 tiles split across ~128 work-groups) and the
    192-channel 3x3 at 32^2."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(C + HW)
    B = 8
    x = torch.randn(B, HW, HW, C, generator=g).to(dtype)
    dz = torch.randn(B, HW, HW, C, generator=g).to(dtype)
    dw = torch.empty((C, C, 3, 3), dtype=torch.float32, device=DEV)
    tdy, tdx = AG._taps(3, 3, 1, 1)
    AG.wgrad(x.to(DEV), dz.to(DEV), tdy, tdx, dw=dw, strides=(C * 9, 9, 1), co_out=C, ci_out=C)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(_nchw(x).double(), (C, C, 3, 3), _nchw(dz).double(), padding=1)
    _check(dw, ref, "wgrad config5")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,H,W,ci,co,k,s,pad", SHAPES + [
    (8, 32, 32, 192, 192, 3, 1, (1, 1, 1, 1)),     # config 5's 192-channel 3x3 (split K over many tiles)
    (2, 16, 16, 64, 200, 3, 1, (1, 1, 1, 1)),      # co = 3 x 64 + 8: a ragged last co block
])
def test_conv_wgrad_fused_bias(dtype, B, H, W, ci, co, k, s, pad):
    """The bias gradient of the same launch (lic_wgrad_args.db: per-split dz column sums finished by
    the split reduce on the tiled 16-bit kernel, the channel-sum pass on the generic / fp32 path)
    against float64 sum_pix dz[pix, n]; then a second launch with accumulate=1 adds both dW and db
    onto what is there."""
    from lic_amd import autograd as AG
    g = torch.Generator().manual_seed(B * 977 + H * 13 + ci + 3 * co + k + s)
    pt, pl, pb, pr = pad
    Ho = (H + pt + pb - k) // s + 1
    Wo = (W + pl + pr - k) // s + 1
    x = torch.randn(B, H, W, ci, generator=g).to(dtype)
    dz = torch.randn(B, Ho, Wo, co, generator=g).to(dtype)
    dw = torch.empty((co, ci, k, k), dtype=torch.float32, device=DEV)
    db = torch.full((co,), float("nan"), dtype=torch.float32, device=DEV)
    tdy, tdx = AG._taps(k, k, pt, pl)
    AG.wgrad(x.to(DEV), dz.to(DEV), tdy, tdx, stride=s, dw=dw, strides=(ci * k * k, k * k, 1), co_out=co,
             ci_out=ci, db=db)
    torch.cuda.synchronize()
    xp = torch.nn.functional.pad(_nchw(x).double(), (pl, pr, pt, pb))
    ref = torch.nn.grad.conv2d_weight(xp, (co, ci, k, k), _nchw(dz).double(), stride=s)
    ref_b = dz.double().sum(dim=(0, 1, 2))
    _check(dw, ref, f"wgrad k{k} s{s} (with db)")
    _check(db, ref_b, f"db k{k} s{s}")
    base_b = torch.randn(co, generator=g)
    db.copy_(base_b)
    AG.wgrad(x.to(DEV), dz.to(DEV), tdy, tdx, stride=s, dw=dw, strides=(ci * k * k, k * k, 1), co_out=co,
             ci_out=ci, db=db, accumulate=True)
    torch.cuda.synchronize()
    _check(dw, 2 * ref, f"wgrad k{k} s{s} accumulate")
    _check(db - base_b.to(DEV), ref_b, f"db k{k} s{s} accumulate")
