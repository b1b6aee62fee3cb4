"""The round-5 16-bit convolution kernel (csrc/conv16.h: transposed MFMA, weights + halo by
LDS-DMA, register epilogue) on the shapes it takes -- stride-1 3x3 / 7x7, >= 16 x 32-pixel maps,
>= 128 tiles -- against torch fp32 on the CPU on the 16-bit-rounded operands (so the bar measures
the kernel's fp32 accumulation and its one output rounding, not the input cast), and against the
generic implicit-GEMM kernel.  Epilogue operand sets (none / r1 / gate g+r1+r2), ragged tiles,
channel-window views and the second destination are covered.  Reference layers: the
Win_noShift_Attention / ResidualBlock 3x3s and the 7x7 of /root/reference/layers/layers.py:87-102,
the ResidualBottleneck 3x3 96->96 of /root/reference/model/net_ga.py:89-103."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
# fp16: one output rounding (2^-11 relative) + accumulation order; bf16: 2^-8 relative
TOL = {torch.float16: 4e-3, torch.bfloat16: 1.2e-2}


def _act(x, dtype):
    from lic_amd.functional import Act
    return Act.from_nchw(x.to(DEV).contiguous(), dtype)


def _rounded(t, dtype):
    return t.to(dtype).float()


def _check(out, ref, dtype, what):
    out = out.float().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"\n[{what}] max err {err:.3e} (scale {scale:.2f})")
    assert torch.isfinite(out).all()
    assert err <= TOL[dtype] * scale, what


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,B,H,W", [
    (192, 192, 3, 32, 64, 64),    # the bench's roofline shape (Win_noShift_Attention 3x3 @ H/4, B=32)
    (192, 192, 3, 16, 64, 64),    # 128 tiles
    (192, 192, 3, 4, 128, 128),   # ResidualBlockWithStride conv2 @ H/2
    (192, 192, 7, 16, 64, 64),    # conv7x7 (tap-row groups)
    (96, 96, 3, 32, 64, 64),      # ResidualBottleneck 3x3 96->96 (96-channel blocks)
    (192, 192, 3, 12, 50, 70),    # ragged tiles in both directions (50 = 3*16+2, 70 = 2*32+6)
    (192, 192, 7, 12, 40, 45),    # ragged 7x7
])
def test_conv16_vs_torch_fp32(dtype, cin, cout, k, B, H, W):
    from lic_amd.layers import Conv2d
    torch.manual_seed(50 + k)
    m = Conv2d(cin, cout, k, 1, k // 2)
    x = torch.randn(B, cin, H, W) * 0.5
    out = m.to(DEV).run(_act(x, dtype)).nchw()
    ref = F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 1, k // 2)
    _check(out, ref, dtype, f"conv{k}x{k} {cin}->{cout} {dtype} B={B} {H}x{W}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,H,W", [(16, 128, 128), (16, 100, 134)])
def test_conv16_stride2_phases_vs_torch_fp32(dtype, B, H, W):
    """ZeroPad2d((1,2,1,2)) + conv5x5 s2 (net_ga.py:277-282): the four input-parity phases (3x3 / 3x2 /
    2x3 / 2x2 taps) accumulate in registers; ragged output (50 x 67 from 100 x 134)."""
    from lic_amd.layers import Conv2d
    torch.manual_seed(55)
    m = Conv2d(192, 192, 5, 2, 0)
    x = torch.randn(B, 192, H, W) * 0.5
    out = m.to(DEV).run(_act(x, dtype), pad=(1, 1, 2, 2)).nchw()
    ref = F.conv2d(F.pad(_rounded(x, dtype), (1, 2, 1, 2)), _rounded(m.weight.detach().cpu(), dtype),
                   m.bias.detach().cpu(), 2)
    _check(out, ref, dtype, f"ZeroPad+conv5x5 s2 {dtype} B={B} {H}x{W}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_conv16_matches_generic(dtype):
    """conv16 vs the generic implicit-GEMM kernel on the same packed operands."""
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    torch.manual_seed(60)
    m = Conv2d(192, 192, 3, 1, 0).to(DEV)
    x = _act(torch.randn(16, 192, 64, 64), dtype)
    pk = m.packed(dtype, (1, 1, 1, 1))
    a = Fn.conv(x, pk).nchw().float()
    b = Fn.conv(x, pk, force_generic=True).nchw().float()
    scale = b.abs().max().item()
    assert (a - b).abs().max().item() <= TOL[dtype] * scale


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_conv16_epilogues_views_dual_store(dtype):
    """The epilogue operand sets the a_model uses on these convs (LeakyReLU; + residual; the
    Win_noShift_Attention gate g*sigmoid(lrelu(acc+b) + r1) + r2), on channel-window views of
    wider buffers, with a second destination."""
    from lic_amd.layers import Conv2d
    from lic_amd.functional import Act
    from lic_amd import _ffi as L
    torch.manual_seed(61)
    B, H, W, C = 16, 64, 64, 192
    m = Conv2d(C, C, 3, 1, 1).to(DEV)
    big = (torch.randn(B, H, W, 3 * C + 64, device=DEV) * 0.5).to(dtype)
    X, R1, G = Act(big, 64, C), Act(big, 64 + C, C), Act(big, 64 + 2 * C, C)
    R2 = Act(big, 0, C)   # overlaps the first channels of X: a read-only view

    def nchw(view):
        return view.t[..., view.c0:view.c0 + view.c].float().permute(0, 3, 1, 2).cpu()

    base = F.conv2d(nchw(X), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 1, 1)
    cases = [
        (dict(act=L.ACT_LRELU), F.leaky_relu(base)),
        (dict(act=L.ACT_LRELU, r1=R1), F.leaky_relu(base) + nchw(R1)),
        (dict(act=L.ACT_LRELU, r1=R1, epi=L.EPI_GATE, g=G, r2=R2),
         nchw(G) * torch.sigmoid(F.leaky_relu(base) + nchw(R1)) + nchw(R2)),
    ]
    for idx, (kw, ref) in enumerate(cases):
        out_buf = torch.zeros(B, H, W, C + 96, device=DEV, dtype=dtype)
        out2 = torch.zeros(B, H, W, C + 32, device=DEV, dtype=dtype)
        m.run(X, out=Act(out_buf, 96, C), y2=Act(out2, 0, C), **kw)
        _check(out_buf[..., 96:].permute(0, 3, 1, 2), ref, dtype, f"epilogue case {idx} {dtype}")
        assert torch.equal(out_buf[..., 96:], out2[..., :C])
        assert out_buf[..., :96].abs().sum().item() == 0 and out2[..., C:].abs().sum().item() == 0


# ---- gemm16 (csrc/gemm16.h): 16-bit 1x1 convolutions on maps of >= 16 K output pixels ----

@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,s,B,H,W", [
    (192, 576, 1, 32, 64, 64),   # WinBasedAttention qkv Linear (three 192-channel blocks)
    (192, 192, 1, 16, 64, 64),   # proj / conv_b 1x1
    (192, 96, 1, 16, 64, 64),    # ResidualBottleneck 192->96 (96-channel blocks)
    (96, 192, 1, 16, 64, 64),    # ResidualBottleneck 96->192 (K = 96)
    (192, 192, 2, 8, 128, 130),  # ResidualBlockWithStride 1x1 s2 skip, ragged (65 columns)
    (192, 192, 1, 7, 50, 47),    # pixel count not a multiple of 32
])
def test_gemm16_vs_torch_fp32(dtype, cin, cout, s, B, H, W):
    from lic_amd.layers import Conv2d
    torch.manual_seed(70 + cin + cout)
    m = Conv2d(cin, cout, 1, s, 0)
    x = torch.randn(B, cin, H, W) * 0.5
    out = m.to(DEV).run(_act(x, dtype)).nchw()
    ref = F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), s)
    _check(out, ref, dtype, f"1x1 s{s} {cin}->{cout} {dtype} B={B} {H}x{W}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm16_epilogues_views(dtype):
    """LeakyReLU / GELU, + residual (the proj shortcut) on channel-window views with a second
    destination."""
    from lic_amd.layers import Conv2d
    from lic_amd.functional import Act
    from lic_amd import _ffi as L
    torch.manual_seed(71)
    B, H, W, C = 8, 64, 64, 192
    m = Conv2d(C, C, 1, 1, 0).to(DEV)
    big = (torch.randn(B, H, W, 2 * C + 32, device=DEV) * 0.5).to(dtype)
    X, R1 = Act(big, 32, C), Act(big, 32 + C, C)

    def nchw(view):
        return view.t[..., view.c0:view.c0 + view.c].float().permute(0, 3, 1, 2).cpu()

    base = F.conv2d(nchw(X), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu())
    for idx, (kw, ref) in enumerate([(dict(act=L.ACT_GELU), F.gelu(base)),
                                     (dict(r1=R1), base + nchw(R1)),
                                     (dict(act=L.ACT_LRELU, r1=R1), F.leaky_relu(base) + nchw(R1))]):
        out_buf = torch.zeros(B, H, W, C + 64, device=DEV, dtype=dtype)
        out2 = torch.zeros(B, H, W, C, device=DEV, dtype=dtype)
        m.run(X, out=Act(out_buf, 64, C), y2=Act(out2), **kw)
        _check(out_buf[..., 64:].permute(0, 3, 1, 2), ref, dtype, f"1x1 epilogue case {idx} {dtype}")
        assert torch.equal(out_buf[..., 64:], out2)
        assert out_buf[..., :64].abs().sum().item() == 0


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("variant", ["compressai", "model_gdn", "model_igdn"])
def test_gemm16_gdn(dtype, variant):
    """GDN / IGDN at 128x128 (the a_model's GDN after ResidualBlockWithStride): x^2 prologue in
    registers + the rsqrt / div / sqrt epilogue with g = x, vs the oracle restatement
    (layers/gdn.py:62-75, model/gdn.py:69-92)."""
    from oracle import ref_cpu as R
    torch.manual_seed(72)
    C = 192
    if variant == "compressai":
        from lic_amd.layers import GDN
        m = GDN(C)
    else:
        from lic_amd.model.gdn import GDN, IGDN
        m = IGDN(C, inverse=True) if variant == "model_igdn" else GDN(C)
    with torch.no_grad():
        m.beta.add_(0.3 * torch.rand(C))
        m.gamma.add_(0.05 * torch.rand(C, C))
    m = m.to(DEV)
    x = torch.randn(2, C, 128, 96) * 2
    out = m.run(_act(x, dtype)).nchw().float().cpu()
    P = {"g." + k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    xr = _rounded(x, dtype)
    ref = R.gdn_compressai(xr, P, "g") if variant == "compressai" else R.gdn_model(xr, P, "g", inverse=(variant == "model_igdn"))
    # the x^2 operand is rounded to the 16-bit type before the MFMA (as every 16-bit kernel does)
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= (1e-2 if dtype == torch.float16 else 3e-2) * scale, (variant, err, scale)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("k,s,act", [(3, 2, "lrelu"), (1, 2, None), (3, 1, None)])
def test_gemm16_image_layers(dtype, k, s, act):
    """The image's first layers (ResidualBlockWithStride(3, 192): conv3x3 s2 + LeakyReLU and the 1x1
    s2 skip, net_ga.py:271) on the 3-channel image zero-padded to 8 channels (Act.zpad): gemm16's
    tap mode, one 16-channel K step per tap with channels 8..15 read as zeros."""
    from lic_amd.layers import Conv2d
    from lic_amd.functional import Act
    from lic_amd import _ffi as L
    torch.manual_seed(73 + k * 10 + s)
    m = Conv2d(3, 192, k, s, k // 2)
    x = torch.rand(8, 3, 128, 128) * 2 - 1
    kw = dict(act=L.ACT_LRELU) if act else {}
    out = m.to(DEV).run(Act.from_nchw(x.to(DEV), dtype, pad16=True), **kw).nchw()
    ref = F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), s, k // 2)
    if act:
        ref = F.leaky_relu(ref)
    _check(out, ref, dtype, f"image layer k{k} s{s} {dtype}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm16_small_map_linear(dtype):
    """1x1 layers on the 16x16 latents (B=32: 8192 pixels, the Swin / WBA Linears of the slice loop)."""
    from lic_amd.layers import Conv2d
    torch.manual_seed(74)
    for ci, co in ((192, 576), (192, 192)):
        m = Conv2d(ci, co, 1, 1, 0)
        x = torch.randn(32, ci, 16, 16) * 0.5
        out = m.to(DEV).run(_act(x, dtype)).nchw()
        ref = F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu())
        _check(out, ref, dtype, f"1x1 {ci}->{co} @16x16 {dtype}")


# ---- conv16s (csrc/conv16s.h): 16-bit stride-1 3x3 / 7x7 on the small maps conv16 does not fill ----

@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,B,H,W", [
    (192, 192, 3, 32, 16, 16),    # Win_noShift_Attention 3x3 @ H/16 (the a_model's 13 latent-map 3x3s)
    (192, 192, 7, 32, 16, 16),    # its conv7x7
    (192, 192, 3, 2, 16, 16),     # few images: 32-channel blocks
    (224, 128, 3, 32, 16, 16),    # slice-loop cc_mean / cc_scale first conv (64-channel blocks)
    (336, 224, 3, 8, 16, 16),     # 21 input chunks: uneven per-wave chunk counts
    (192, 192, 3, 4, 32, 32),     # a 32x32 map with too few tiles for conv16
    (192, 192, 3, 3, 13, 21),     # ragged tiles (13 = 3*4+1 rows, 21 = 16+5 columns)
    (192, 192, 7, 5, 9, 30),      # ragged 7x7
    (128, 32, 3, 16, 16, 16),     # narrow output (one 32-channel block)
    (128, 512, 1, 8, 16, 16),     # 1x1: slice-loop Swin MLP Linears (training batch), 64-channel blocks
    (512, 128, 1, 8, 16, 16),     # 1x1: 32 input chunks over 4 waves
    (64, 128, 1, 8, 16, 16),      # 1x1: ResidualUnit conv 64->128 (4 chunks: one per wave)
    (240, 128, 1, 32, 16, 16),    # 1x1: SWAtten in_conv (15 chunks), the inference batch (8 K pixels)
    (128, 64, 1, 3, 13, 21),      # 1x1: ragged tiles
])
def test_conv16s_vs_torch_fp32(dtype, cin, cout, k, B, H, W):
    from lic_amd.layers import Conv2d
    torch.manual_seed(80 + k + cin)
    m = Conv2d(cin, cout, k, 1, k // 2)
    x = torch.randn(B, cin, H, W) * 0.5
    out = m.to(DEV).run(_act(x, dtype)).nchw()
    ref = F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 1, k // 2)
    _check(out, ref, dtype, f"conv16s conv{k}x{k} {cin}->{cout} {dtype} B={B} {H}x{W}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_conv16s_epilogues_views_dual_store(dtype):
    """The latent-map Win_noShift_Attention epilogues (LeakyReLU; + residual; the gate
    g*sigmoid(lrelu(acc+b) + r1) + r2) on channel-window views with a second destination, and the
    generic implicit-GEMM kernel on the same packed operands."""
    from lic_amd.layers import Conv2d
    from lic_amd.functional import Act
    import lic_amd.functional as Fn
    from lic_amd import _ffi as L
    torch.manual_seed(62)
    B, H, W, C = 32, 16, 16, 192
    m = Conv2d(C, C, 3, 1, 1).to(DEV)
    big = (torch.randn(B, H, W, 3 * C + 64, device=DEV) * 0.5).to(dtype)
    X, R1, G = Act(big, 64, C), Act(big, 64 + C, C), Act(big, 64 + 2 * C, C)
    R2 = Act(big, 0, C)

    def nchw(view):
        return view.t[..., view.c0:view.c0 + view.c].float().permute(0, 3, 1, 2).cpu()

    base = F.conv2d(nchw(X), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 1, 1)
    cases = [
        (dict(act=L.ACT_LRELU), F.leaky_relu(base)),
        (dict(act=L.ACT_LRELU, r1=R1), F.leaky_relu(base) + nchw(R1)),
        (dict(act=L.ACT_LRELU, r1=R1, epi=L.EPI_GATE, g=G, r2=R2),
         nchw(G) * torch.sigmoid(F.leaky_relu(base) + nchw(R1)) + nchw(R2)),
    ]
    for idx, (kw, ref) in enumerate(cases):
        out_buf = torch.zeros(B, H, W, C + 96, device=DEV, dtype=dtype)
        out2 = torch.zeros(B, H, W, C + 32, device=DEV, dtype=dtype)
        m.run(X, out=Act(out_buf, 96, C), y2=Act(out2, 0, C), **kw)
        _check(out_buf[..., 96:].permute(0, 3, 1, 2), ref, dtype, f"conv16s epilogue case {idx} {dtype}")
        assert torch.equal(out_buf[..., 96:], out2[..., :C])
        assert out_buf[..., :96].abs().sum().item() == 0 and out2[..., C:].abs().sum().item() == 0
    pk = m.packed(dtype, (1, 1, 1, 1))
    a = Fn.conv(X, pk).nchw().float()
    b = Fn.conv(X, pk, force_generic=True).nchw().float()
    assert (a - b).abs().max().item() <= TOL[dtype] * b.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm16_gdn_residual(dtype):
    """GDN + skip (ResidualBlockWithStride, net_ga.py:68-86: gdn(conv2(...)) + skip(x)) as one launch:
    the GDN epilogue with the residual operand."""
    from lic_amd.layers import GDN
    from lic_amd.functional import Act
    import lic_amd.functional as Fn
    from lic_amd._ffi import EPI_GDN_RSQRT, PRO_SQUARE
    from oracle import ref_cpu as R
    torch.manual_seed(75)
    C = 192
    m = GDN(C)
    with torch.no_grad():
        m.beta.add_(0.3 * torch.rand(C))
        m.gamma.add_(0.05 * torch.rand(C, C))
    m = m.to(DEV)
    x = torch.randn(4, C, 128, 96) * 2
    r = torch.randn(4, C, 128, 96)
    out = Fn.gdn(_act(x, dtype), m.packed(dtype), EPI_GDN_RSQRT, None, _act(r, dtype)).nchw().float().cpu()
    P = {"g." + k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    xr, rr = _rounded(x, dtype), _rounded(r, dtype)
    ref = R.gdn_compressai(xr, P, "g") + rr
    err = (out - ref).abs().max().item()
    assert err <= (1e-2 if dtype == torch.float16 else 3e-2) * ref.abs().max().item(), err
    # g another tensor than the input (the register-g variant does not apply): g * rsqrt(beta + gamma x^2) + r1
    y = torch.randn(4, C, 128, 96)
    out2 = Fn.conv(_act(x, dtype), m.packed(dtype), epi=EPI_GDN_RSQRT, g=_act(y, dtype), r1=_act(r, dtype),
                   prologue=PRO_SQUARE).nchw().float().cpu()
    beta = R.nnp_forward(P["g.beta"], P["g.beta_reparam.lower_bound.bound"], P["g.beta_reparam.pedestal"])
    gamma = R.nnp_forward(P["g.gamma"], P["g.gamma_reparam.lower_bound.bound"], P["g.gamma_reparam.pedestal"])
    ref2 = _rounded(y, dtype) * torch.rsqrt(F.conv2d(xr ** 2, gamma.reshape(C, C, 1, 1), beta)) + rr
    err2 = (out2 - ref2).abs().max().item()
    assert err2 <= (1e-2 if dtype == torch.float16 else 3e-2) * ref2.abs().max().item(), err2


# ---- wba16 (csrc/wba16.hip): 16-bit qkv Linear + window attention in one launch ----

@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
# (16|32, 64, 64): 1024 / 2048 windows, more than the persistent grid's workgroups, so every workgroup walks
# several windows (next-window prefetch, LDS reuse without a barrier, per-window mask: ADVICE r5)
@pytest.mark.parametrize("B,H,W,shift", [(4, 64, 64, 4), (2, 32, 48, 0), (3, 16, 24, 4), (16, 64, 64, 4),
                                         (32, 64, 64, 0)])
def test_wba16_matches_unfused(dtype, B, H, W, shift):
    """The fused launch against the two-launch path (qkv Linear -> win_attn, whose own parity against
    the oracle is tests/test_gpu_attn.py) on the same operands: WinBasedAttention, reference
    layers/win_attention.py:85-116 + 154-209, with the region mask of the shifted windows at the last
    window row / column; and the whole block (proj + shortcut) through the module."""
    import lic_amd.functional as Fn
    from lic_amd.functional import Act
    from lic_amd.layers.win_attention import WinBasedAttention
    torch.manual_seed(90 + H + shift)
    m = WinBasedAttention(dim=192, num_heads=8, window_size=8, shift_size=shift).to(DEV)
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0, 0.5)
    x = Act.from_nchw((torch.randn(B, 192, H, W) * 0.7).to(DEV), dtype)
    att = m.attn
    args = (8, 8, shift, att.relative_position_bias_table, 8, 1, 1 if shift > 0 else 0, float(att.scale))
    fused = Fn.wba16_qkv_attn(x, att.qkv.packed(dtype), *args).nchw().float()
    qkv = att.qkv.run(x)
    unfused = Fn.win_attn(qkv, 192, 8, 8, shift, att.relative_position_bias_table, 8, 1, 1 if shift > 0 else 0,
                          False, float(att.scale)).nchw().float()
    scale = unfused.abs().max().item()
    # same operands and rounding points; the qkv accumulation order differs (fp32 sums of 192 products)
    assert (fused - unfused).abs().max().item() <= 2 * TOL[dtype] * scale
    # the whole block (proj + shortcut) through the module against the three-launch path
    blk = m.run(x).nchw().float()
    ref_blk = att.proj.run(Act.from_nchw(unfused, dtype), r1=x).nchw().float()
    assert (blk - ref_blk).abs().max().item() <= 4 * TOL[dtype] * ref_blk.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_conv16_gelu_96(dtype):
    """ResidualBottleneck's 3x3 96->96 + GELU (net_ga.py:89-103): conv16's 96-channel register epilogue."""
    from lic_amd.layers import Conv2d
    from lic_amd import _ffi as L
    torch.manual_seed(63)
    m = Conv2d(96, 96, 3, 1, 1)
    x = torch.randn(32, 96, 64, 64) * 0.5
    out = m.to(DEV).run(_act(x, dtype), act=L.ACT_GELU).nchw()
    ref = F.gelu(F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 1, 1))
    _check(out, ref, dtype, f"conv3x3 96->96 + GELU {dtype}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,H,W", [(32, 64, 64), (16, 128, 128), (12, 70, 100)])
def test_conv16_stride2_3x3(dtype, B, H, W):
    """ResidualBlockWithStride's conv3x3 s2 pad 1 (net_ga.py:68-86) on conv16's input-parity phases
    (2x2 / 2x1 / 1x2 / 1x1 taps), 96- and 192-channel blocks, ragged output (35 x 50 from 70 x 100)."""
    from lic_amd.layers import Conv2d
    from lic_amd import _ffi as L
    torch.manual_seed(64 + H)
    m = Conv2d(192, 192, 3, 2, 1)
    x = torch.randn(B, 192, H, W) * 0.5
    out = m.to(DEV).run(_act(x, dtype), act=L.ACT_LRELU).nchw()
    ref = F.leaky_relu(F.conv2d(_rounded(x, dtype), _rounded(m.weight.detach().cpu(), dtype), m.bias.detach().cpu(), 2, 1))
    _check(out, ref, dtype, f"conv3x3 s2 {dtype} B={B} {H}x{W}")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,stride,B,H,W", [
    (192, 192, 3, 1, 32, 64, 64),      # conv16 3x3, 192-channel blocks
    (96, 96, 3, 1, 32, 64, 64),        # conv16 96-channel blocks
    (192, 192, 5, 2, 32, 128, 128),    # conv16 ZeroPad + 5x5 s2 phases
    (192, 192, 7, 1, 32, 64, 64),      # conv16 7x7
    (192, 192, 3, 1, 32, 16, 16),      # conv16s 3x3 @16^2
    (224, 128, 3, 1, 32, 16, 16),      # conv16s (slice-loop cc conv)
    (192, 192, 7, 1, 32, 16, 16),      # conv16s 7x7
])
def test_frag16_weights_bit_identical(dtype, cin, cout, k, stride, B, H, W):
    """conv16 / conv16s with the weights in MFMA-fragment order (functional.frag16_weights, built on a pack's
    second use; include/lic.h wgt_split) give the same bits as the [copad][ntaps][cpad] rows: only the load
    addresses differ."""
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    torch.manual_seed(70 + k + H)
    m = Conv2d(cin, cout, k, stride, k // 2 if stride == 1 else 0).to(DEV)
    x = _act(torch.randn(B, cin, H, W) * 0.5, dtype)
    pad = None if stride == 1 else (1, 1, 2, 2)
    y_rows = m.run(x, pad=pad).t.clone()
    pk = m.packed(x.dtype, pad if pad is not None else (m.padding[0],) * 4)
    assert Fn.frag16_weights(pk) is not None        # second use: the fragment-order copy exists now
    y_frag = m.run(x, pad=pad).t
    assert torch.equal(y_rows, y_frag)
