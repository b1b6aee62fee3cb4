"""Per-kernel parity of the HIP path (through the C ABI) against the CPU oracle /
fp32 torch CPU on the same seeded inputs.  Tolerances: fp32 path rtol/atol 1e-4
(exact-fp32 MFMA vs oneDNN summation order); fp16 path 2e-2 relative to the
tensor's scale; quantised symbols bit-exact given identical (y, mu)."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _P(module, prefix=""):
    return {(prefix + "." + k if prefix else k): v.detach().float().cpu() for k, v in module.state_dict().items()}


def _close(out, ref, dtype, rtol=1e-4, atol=1e-4):
    out = out.float().cpu()
    ref = ref.float().cpu()
    if dtype != torch.float32:   # 16-bit activations: fp16 2e-2, bf16 4e-2 of the scale
        scale = ref.abs().max().item() + 1e-6
        err = (out - ref).abs().max().item()
        tol = 2e-2 if dtype == torch.float16 else 4e-2
        assert err <= tol * scale, f"{dtype} max err {err} vs scale {scale}"
    else:
        torch.testing.assert_close(out, ref, rtol=rtol, atol=atol)


def _act(x, dtype):
    from lic_amd.functional import Act
    return Act.from_nchw(x.to(DEV).contiguous(), dtype)


DTYPES = [torch.float32, torch.float16, torch.bfloat16]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cin,cout,k,s,pad,H", [
    (192, 192, 3, 1, (1, 1, 1, 1), 16),   # MFMA, BN=192
    (96, 96, 3, 1, (1, 1, 1, 1), 12),     # BN=96
    (192, 96, 1, 1, (0, 0, 0, 0), 9),
    (192, 192, 5, 2, (1, 1, 2, 2), 16),   # ZeroPad2d((1,2,1,2)) + conv5x5 s2
    (64, 192, 7, 1, (3, 3, 3, 3), 8),
    (48, 224, 3, 1, (1, 1, 1, 1), 8),     # K tail (48 % 32), co pad to 256
    (3, 192, 3, 2, (1, 1, 1, 1), 17),     # direct kernel (Cin=3)
    (16, 320, 3, 1, (1, 1, 1, 1), 5),
])
def test_conv2d(dtype, cin, cout, k, s, pad, H):
    from lic_amd.layers import Conv2d
    torch.manual_seed(0)
    m = Conv2d(cin, cout, k, s, 0).to(DEV)
    x = torch.randn(2, cin, H, H + 1)
    out = m.run(_act(x, dtype), pad=pad).nchw()
    ref = F.conv2d(F.pad(x, (pad[1], pad[3], pad[0], pad[2])), m.weight.cpu(), m.bias.cpu(), s)
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv_direct_matches_mfma(dtype):
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    torch.manual_seed(1)
    m = Conv2d(64, 128, 3, 1, 1).to(DEV)
    x = _act(torch.randn(2, 64, 10, 10), dtype)
    pk = m.packed(dtype)
    a = Fn.conv(x, pk)
    b = Fn.conv(x, pk, force_direct=True)
    _close(a.nchw(), b.nchw(), dtype, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv_epilogues(dtype):
    from lic_amd.layers import Conv2d
    from lic_amd import _ffi as L
    torch.manual_seed(2)
    m = Conv2d(64, 64, 3, 1, 1).to(DEV)
    x = torch.randn(2, 64, 8, 8)
    r = torch.randn(2, 64, 8, 8)
    g = torch.randn(2, 64, 8, 8)
    base = F.conv2d(x, m.weight.cpu(), m.bias.cpu(), 1, 1)
    X, Rr, G = _act(x, dtype), _act(r, dtype), _act(g, dtype)
    cases = [
        (dict(act=L.ACT_GELU), F.gelu(base)),
        (dict(act=L.ACT_RELU, r1=Rr), F.relu(base) + r),
        (dict(act=L.ACT_LRELU, slope=0.2, r1=Rr), F.leaky_relu(base, 0.2) + r),
        (dict(act=L.ACT_LRELU, r1=Rr, epi=L.EPI_GATE, g=G, r2=X), g * torch.sigmoid(F.leaky_relu(base) + r) + x),
        (dict(epi=L.EPI_HALF_TANH, r2=Rr), r + 0.5 * torch.tanh(base)),
        (dict(act=L.ACT_RELU, r1=Rr, epi=L.EPI_RES_ACT), F.relu(base + r)),
        (dict(act=L.ACT_ROUND), torch.round(base)),
    ]
    for kw, ref in cases:
        out = m.run(X, **kw).nchw()
        if kw.get("act") == L.ACT_ROUND and dtype != torch.float16:
            # rounding is exact given the same pre-activation; allow values near .5 flipped by
            # summation order (fp32) or by bf16's 8-bit operands (a few %)
            assert (out.cpu() - ref).abs().max().item() <= 1.0
            assert (out.cpu() != ref).float().mean().item() < (1e-3 if dtype == torch.float32 else 5e-2)
            continue
        _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv_views_and_dual_store(dtype):
    """Channel-window views (concat buffers) for input, output, residual and a second destination."""
    from lic_amd.layers import Conv2d
    from lic_amd.functional import Act
    torch.manual_seed(3)
    m = Conv2d(48, 48, 3, 1, 1).to(DEV)
    big = torch.randn(2, 7, 9, 240, device=DEV).to(dtype)
    X = Act(big, 96, 48)
    out_buf = torch.zeros(2, 7, 9, 384, device=DEV, dtype=dtype)
    out2 = torch.zeros(2, 7, 9, 336, device=DEV, dtype=dtype)
    R1 = Act(big, 16, 48)
    m.run(X, out=Act(out_buf, 192, 48), r1=R1, y2=Act(out2, 240, 48))
    x = big[..., 96:144].float().permute(0, 3, 1, 2).cpu()
    ref = F.conv2d(x, m.weight.cpu(), m.bias.cpu(), 1, 1) + big[..., 16:64].float().permute(0, 3, 1, 2).cpu()
    _close(out_buf[..., 192:240].permute(0, 3, 1, 2), ref, dtype)
    _close(out2[..., 240:288].permute(0, 3, 1, 2), ref, dtype)
    assert out_buf[..., :192].abs().sum().item() == 0 and out_buf[..., 240:].abs().sum().item() == 0


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("ci,co,k,s,p,op,prepad,H", [(192, 192, 5, 2, 3, 1, (1, 1), 8), (192, 16, 5, 2, 3, 1, (1, 1), 6),
                                                      (512, 256, 5, 2, 2, 1, (0, 0), 4), (384, 192, 1, 1, 0, 0, (0, 0), 5)])
def test_conv_transpose(dtype, ci, co, k, s, p, op, prepad, H):
    from lic_amd.layers import ConvTranspose2d
    torch.manual_seed(4)
    m = ConvTranspose2d(ci, co, k, s, p, output_padding=op).to(DEV)
    x = torch.randn(2, ci, H, H)
    out = m.run(_act(x, dtype), prepad=prepad).nchw()
    ref = F.conv_transpose2d(F.pad(x, (prepad[1], 0, prepad[0], 0)), m.weight.cpu(), m.bias.cpu(), s, p, op)
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_subpel_shuffle(dtype):
    from lic_amd.layers import subpel_conv3x3
    torch.manual_seed(5)
    m = subpel_conv3x3(64, 32, 2).to(DEV)
    x = torch.randn(2, 64, 5, 6)
    out = m[0].run(_act(x, dtype), shuffle=True).nchw()
    ref = F.pixel_shuffle(F.conv2d(x, m[0].weight.cpu(), m[0].bias.cpu(), 1, 1), 2)
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("variant", ["model_gdn", "model_igdn", "compressai"])
def test_gdn(dtype, variant):
    torch.manual_seed(6)
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
    x = torch.randn(2, C, 6, 7) * 2
    out = m.run(_act(x, dtype)).nchw()
    P = _P(m, "g")
    if variant == "compressai":
        ref = R.gdn_compressai(x, P, "g")
    else:
        ref = R.gdn_model(x, P, "g", inverse=(variant == "model_igdn"))
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("C,heads,ws,shift,H,W", [(192, 8, 8, 4, 16, 16), (192, 8, 4, 2, 8, 12), (64, 8, 4, 2, 4, 4),
                                                  (512, 8, 2, 1, 4, 4), (96, 8, 4, 2, 16, 8), (128, 8, 8, 0, 16, 8)])
def test_win_based_attention(dtype, C, heads, ws, shift, H, W):
    from lic_amd.layers import WinBasedAttention
    torch.manual_seed(7)
    m = WinBasedAttention(C, heads, ws, shift)
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0, 0.05)
    m = m.to(DEV)
    x = torch.randn(2, C, H, W)
    out = m.run(_act(x, dtype)).nchw()
    ref = R.win_based_attention(x, _P(m, "w"), "w", heads, ws, shift)
    _close(out, ref, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_swin_block_1(dtype):
    from lic_amd.model.net_ga import SwinBlock
    from lic_amd.functional import Act
    torch.manual_seed(8)
    m = SwinBlock(128, 128, 16, 8, 0)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "ln" not in n:
                p.normal_(0, 0.05)
    m = m.to(DEV)
    x = torch.randn(2, 128, 16, 16)
    out = m.run(_act(x, dtype)).nchw()
    ref = R.swin_block(x, _P(m, "s"), "s", 16, 8)
    _close(out, ref, dtype, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("dtype", DTYPES)
def test_swatten(dtype):
    from lic_amd.model.net_ga import SWAtten
    torch.manual_seed(9)
    m = SWAtten(240, 240, 16, 8, 0, inter_dim=128)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "ln" not in n:
                p.normal_(0, 0.04)
    m = m.to(DEV)
    x = torch.randn(2, 240, 16, 16)
    out = m.run(_act(x, dtype)).nchw()
    ref = R.swatten(x, _P(m, "a"), "a")
    _close(out, ref, dtype, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("dtype", DTYPES)
def test_win_noshift_attention(dtype):
    from lic_amd.layers import Win_noShift_Attention
    from lic_amd.model.net_ga import weight_init
    torch.manual_seed(10)
    m = Win_noShift_Attention(192, 8, 8, 4)
    m.apply(weight_init)
    m = m.to(DEV)
    x = torch.randn(1, 192, 16, 16)
    out = m.run(_act(x, dtype)).nchw()
    ref = R.win_noshift_attention(x, _P(m, "n"), "n", 8, 8, 4)
    _close(out, ref, dtype, rtol=3e-4, atol=3e-4)


@pytest.mark.parametrize("dtype", DTYPES)
def test_layernorm(dtype):
    import lic_amd.functional as Fn
    torch.manual_seed(11)
    x = torch.randn(2, 5, 7, 128) * 3 + 1
    w = torch.randn(128)
    b = torch.randn(128)
    out = Fn.layernorm(Fn.Act(x.to(DEV).to(dtype).contiguous()), w.to(DEV), b.to(DEV), 1e-5)
    ref = F.layer_norm(x.to(dtype).float(), (128,), w, b)
    _close(out.t, ref, dtype)


def test_rate_symbols_bit_exact_given_same_inputs():
    """The quantised symbol indices are bit-exact given identical (y, mu): the kernel's
    rint(y - mu) equals the oracle's round_half_even on the same fp32 values."""
    import lic_amd.functional as Fn
    torch.manual_seed(12)
    B, H, W, C = 2, 8, 8, 48
    y = torch.randn(B, H, W, C) * 5
    mu = torch.randn(B, H, W, C)
    # force exact .5 ties and near-ties
    y[0, 0, 0, :8] = mu[0, 0, 0, :8] + torch.tensor([0.5, 1.5, -0.5, -2.5, 2.5, 0.4999999, 3.5, -3.5])
    sc = torch.rand(B, H, W, C) * 3
    Y, MU, SC = (Fn.Act(t.to(DEV).contiguous()) for t in (y, mu, sc))
    sym = torch.empty(B, H, W, C, dtype=torch.int32, device=DEV)
    lik = torch.empty(B, H, W, C, dtype=torch.float32, device=DEV)
    yq = Fn.Act.empty(B, H, W, C, torch.float32, DEV)
    parts = torch.zeros(1024, dtype=torch.float64, device=DEV)
    n = Fn.gauss_rate(Y, MU, SC, parts, 0, yq=yq, symbols=Fn.Act(sym), likelihood=Fn.Act(lik))
    ref_sym = R.symbols(y, mu)
    assert torch.equal(sym.cpu(), ref_sym)
    ref_yq = R.quantize_dequantize(y, mu)
    assert torch.equal(yq.t.cpu(), ref_yq)
    ref_lik = R.gaussian_likelihood(ref_yq, sc, mu)
    torch.testing.assert_close(lik.cpu(), ref_lik, rtol=2e-6, atol=1e-9)
    out = torch.empty(1, dtype=torch.float32, device=DEV)
    Fn.bpp_finalize(parts, n, B * H * W * 16, out)
    ref_bpp = torch.sum(torch.log(ref_lik)) / (-math.log(2) * B * H * W * 16)
    assert abs(out.item() - ref_bpp.item()) <= 1e-5 * max(1.0, abs(ref_bpp.item()))


def test_quantize_median():
    import lic_amd.functional as Fn
    torch.manual_seed(13)
    z = torch.randn(2, 4, 4, 192) * 4
    m = torch.randn(192)
    out = Fn.quantize_median(Fn.Act(z.to(DEV)), m.to(DEV))
    assert torch.equal(out.t.cpu(), torch.round(z - m) + m)


def test_syntax_recon_and_psnr():
    import lic_amd.functional as Fn
    torch.manual_seed(14)
    B, H, W = 2, 32, 24
    xt = torch.randn(B, H, W, 16)
    wg = torch.randn(B, 1, 1, 48) * 0.3
    x = torch.rand(B, 3, H, W) * 2 - 1
    x_rec = torch.empty(B, 3, H, W, device=DEV)
    parts = torch.empty(B * 2, dtype=torch.float64, device=DEV)
    Fn.syntax_recon(Fn.Act(xt.to(DEV)), Fn.Act(wg.to(DEV)), x.to(DEV), x_rec, parts, 2)
    v_mse = torch.empty(B, device=DEV)
    v_psnr = torch.empty(1, device=DEV)
    Fn.psnr_finalize(parts, B, 2, 3.0 * H * W, v_mse, v_psnr)
    xtil = xt.permute(0, 3, 1, 2)
    ref = torch.clamp(torch.tanh(R.batch_conv(wg.view(B, 3, 16, 1, 1), xtil)), -1, 1)
    torch.testing.assert_close(x_rec.cpu(), ref, rtol=1e-5, atol=1e-5)
    gt = torch.round((x + 1) * 127.5)
    xh = torch.round(torch.clamp((ref + 1) * 127.5, 0, 255))
    ref_mse = torch.mean((xh - gt) ** 2, [1, 2, 3])
    torch.testing.assert_close(v_mse.cpu(), ref_mse, rtol=1e-4, atol=1e-3)
    ref_psnr = torch.mean(20 * torch.log10(255 / torch.sqrt(ref_mse)))
    assert abs(v_psnr.item() - ref_psnr.item()) < 1e-3


def test_loud_failure_on_bad_args():
    """Invalid launches report through lic_last_error instead of running anything."""
    import lic_amd.functional as Fn
    from lic_amd._ffi import LicError
    from lic_amd.layers import Conv2d
    m = Conv2d(16, 16, 3, 1, 1).to(DEV)
    x = Fn.Act(torch.randn(1, 4, 4, 8, device=DEV))
    with pytest.raises(ValueError):
        m.run(x)  # channel mismatch caught on the host
    a = Fn.Act(torch.randn(1, 6, 6, 24, device=DEV))
    with pytest.raises(LicError):
        Fn.win_attn(a, 8, 3, 4, 0, torch.zeros(49, 3, device=DEV), 3, 1, 0, False, 1.0)  # 6 % 4 != 0


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cin,cout,k,s,pad,B,H", [
    (192, 192, 3, 1, (1, 1, 1, 1), 16, 64),   # Win_noShift_Attention conv3x3 @ H/4
    (192, 192, 7, 1, (3, 3, 3, 3), 16, 64),   # conv7x7 (tap groups)
    (192, 192, 5, 2, (1, 1, 2, 2), 8, 128),   # ZeroPad2d((1,2,1,2)) + conv5x5 s2
    (192, 192, 3, 2, (1, 1, 1, 1), 8, 96),    # RBWS conv1 (stride 2), ragged tiles (96/2=48)
    (96, 96, 3, 1, (1, 1, 1, 1), 16, 50),     # ragged tile edges, BN=128 pad
    (64, 64, 3, 1, (1, 1, 1, 1), 8, 256),     # HAN conv3x3 @ full res (fp16: 32x16 px x 64 ch tiles)
    (64, 64, 3, 1, (1, 1, 1, 1), 9, 250),     # same, ragged 32x16 tiles
    # the bench's configuration (B=32 at 64x64 -> fp16 32x16-px x 192-ch tiles, conv.hip)
    (192, 192, 3, 1, (1, 1, 1, 1), 32, 64),
    (192, 192, 7, 1, (3, 3, 3, 3), 32, 64),
    (192, 192, 3, 1, (1, 1, 1, 1), 28, 56),   # ragged 32x16 tiles (56 = 32 + 24, 56 = 3*16 + 8)
])
def test_conv_halo_matches_generic(dtype, cin, cout, k, s, pad, B, H):
    """The spatial-tile (halo) kernel and the generic implicit-GEMM kernel agree."""
    from lic_amd.layers import Conv2d
    import lic_amd.functional as Fn
    torch.manual_seed(15)
    m = Conv2d(cin, cout, k, s, 0).to(DEV)
    x = _act(torch.randn(B, cin, H, H), dtype)
    pk = m.packed(dtype, pad)
    a = Fn.conv(x, pk)
    b = Fn.conv(x, pk, force_generic=True)
    _close(a.nchw(), b.nchw(), dtype, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv_transpose_halo_matches_cpu(dtype):
    """s_model's ZeroPad2d((1,0,1,0)) + ConvTranspose2d(5, 2, 3, op=1) at a size that takes the halo kernel."""
    from lic_amd.layers import ConvTranspose2d
    torch.manual_seed(16)
    m = ConvTranspose2d(192, 192, 5, 2, 3, output_padding=1).to(DEV)
    x = torch.randn(8, 192, 32, 32)
    out = m.run(_act(x, dtype), prepad=(1, 1)).nchw()
    ref = F.conv_transpose2d(F.pad(x, (1, 0, 1, 0)), m.weight.cpu(), m.bias.cpu(), 2, 3, 1)
    _close(out, ref, dtype)


def _big_tile_selected(B, H, co=192):
    """Mirror of conv.hip's fp16 tile choice: 32x16 px x 192 ch when the grid has >= 200
    such workgroups (stride 1, co % 192 == 0, map taller than 16)."""
    return co % 192 == 0 and H > 16 and B * (-(-H // 32)) * (-(-H // 16)) * (co // 192) >= 200


@pytest.mark.parametrize("k,B,H", [(3, 32, 64), (7, 32, 64), (3, 28, 56)])
def test_conv_halo_32x16_tile_fp16_vs_torch_fp32(k, B, H):
    """The headline kernel configuration (fp16 conv_halo_kernel<32,16,192>, the bench's
    roofline kernel) against torch fp32 on the CPU: fp16 operands, fp32 accumulation."""
    from lic_amd.layers import Conv2d
    assert _big_tile_selected(B, H)
    torch.manual_seed(17)
    m = Conv2d(192, 192, k, 1, k // 2)
    x = torch.randn(B, 192, H, H) * 0.5
    out = m.to(DEV).run(_act(x, torch.float16)).nchw().float().cpu()
    # reference on the fp16-rounded operands, so the bar measures the kernel, not the cast
    ref = F.conv2d(x.half().float(), m.weight.detach().cpu().half().float(), m.bias.detach().cpu(), 1, k // 2)
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"\n[conv{k}x{k} fp16 32x16 tile B={B} {H}x{H}] max err {err:.3e} (scale {scale:.2f})")
    assert err <= 4e-3 * scale
