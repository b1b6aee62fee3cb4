"""GPU parity of the window-attention kernels (lic_win_attn_fwd).

The 8x8-window MFMA kernel (csrc/attention_mfma.hip) and the VALU kernel
(csrc/attention.hip, force_valu=1) are both checked against a plain PyTorch fp32
restatement of the fused op: roll(-shift) + window_partition + softmax(q k^T * scale
+ bias + mask) v + window_reverse + roll(+shift), with the masks built by the oracle
(layers/win_attention.py:160-181 WBA, model/Block_unet.py:197-214 WMSA).
"""
import pytest
import torch

from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _attn_ref(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale):
    """qkv: [B, H, W, >=3C] fp32; table [(2ws-1)^2, heads]."""
    B, H, W, _ = qkv.shape
    d = C // heads
    x = torch.roll(qkv[..., :3 * C], shifts=(-shift, -shift), dims=(1, 2)) if shift else qkv[..., :3 * C]
    win = R.window_partition(x.contiguous(), ws).view(-1, ws * ws, 3 * C)  # [B*nw, N, 3C]
    q = win[..., :C].view(-1, ws * ws, heads, d).transpose(1, 2)
    k = win[..., C:2 * C].view(-1, ws * ws, heads, d).transpose(1, 2)
    v = win[..., 2 * C:].view(-1, ws * ws, heads, d).transpose(1, 2)
    s = (q @ k.transpose(-2, -1)) * scale if scale_after else (q * scale) @ k.transpose(-2, -1)
    rpi = R.relative_position_index(ws).view(-1)
    s = s + table[rpi].view(ws * ws, ws * ws, heads).permute(2, 0, 1)[None]
    nw = (H // ws) * (W // ws)
    if mask_kind == 1:
        m = R.wba_mask(H, W, ws, shift)  # [nw, N, N]
        s = (s.view(B, nw, heads, ws * ws, ws * ws) + m[None, :, None]).view_as(s)
    elif mask_kind == 2:
        m = R.wmsa_mask(H // ws, W // ws, ws, shift)
        s = s.view(B, nw, heads, ws * ws, ws * ws).masked_fill(m[None, :, None], float("-inf")).view_as(s)
    o = torch.softmax(s, dim=-1) @ v  # [B*nw, heads, N, d]
    o = o.transpose(1, 2).reshape(-1, ws, ws, C)
    o = R.window_reverse(o, ws, H, W)
    return torch.roll(o, shifts=(shift, shift), dims=(1, 2)) if shift else o


def _run(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale, dtype, force_valu):
    import lic_amd.functional as Fn
    a = Fn.Act(qkv.to(DEV).to(dtype).contiguous())
    tab = table.to(DEV).contiguous()
    out = Fn.win_attn(a, C, heads, ws, shift, tab, heads, 1, mask_kind, scale_after, scale, force_valu=force_valu)
    torch.cuda.synchronize()
    return out.t[..., :C].float().cpu()


CASES = [
    # C, heads, ws, shift, H, W, mask_kind, scale_after
    (192, 8, 8, 4, 16, 16, 1, False),   # Win_noShift_Attention ws 8 (net_ga.py:157), d = 24
    (192, 8, 8, 2, 16, 24, 1, False),   # synthesis ws 8 shift 2 (net_ga.py:199)
    (128, 8, 8, 0, 16, 8, 0, True),     # SwinBlock 'W' (d = 16)
    (128, 8, 8, 4, 24, 16, 2, True),    # SwinBlock 'SW' (WMSA mask)
    (256, 8, 8, 4, 16, 16, 2, True),    # d = 32
    (48, 6, 8, 4, 8, 16, 1, False),     # d = 8, heads not a multiple of 4
    (96, 4, 8, 0, 8, 8, 0, False),      # d = 24, single window
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("C,heads,ws,shift,H,W,mask_kind,scale_after", CASES)
def test_mfma_attention_matches_reference(dtype, C, heads, ws, shift, H, W, mask_kind, scale_after):
    g = torch.Generator().manual_seed(C * 7 + H + W + shift)
    B = 2
    qkv = torch.randn(B, H, W, 3 * C, generator=g)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    scale = (C // heads) ** -0.5
    qkv_q = qkv.to(dtype).float()
    ref = _attn_ref(qkv_q, C, heads, ws, shift, table, mask_kind, scale_after, scale)
    out = _run(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale, dtype, False)
    valu = _run(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale, dtype, True)
    if dtype == torch.float32:
        torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(out, valu, rtol=1e-4, atol=1e-4)
    else:
        # 16-bit operands and 16-bit probabilities into the PV product, fp32 accumulation
        tol = 1e-2 if dtype == torch.float16 else 3e-2
        assert (out - ref).abs().max().item() <= tol * (ref.abs().max().item() + 1e-6)
        assert (out - valu).abs().max().item() <= tol * (ref.abs().max().item() + 1e-6)


@pytest.mark.parametrize("C,heads,ws,shift,H,W,mask_kind,scale_after", CASES)
def test_split_attention_fp32_grade(C, heads, ws, shift, H, W, mask_kind, scale_after):
    """fp32 data under split mode 2 (fp32x6: Q, K, V, P as three bf16 parts, 6 part products)
    against a float64 restatement: as close as the exact fp32 MFMA kernel (both errors at the
    fp32 rounding level, 2e-6 of the output scale)."""
    import lic_amd.functional as Fn
    g = torch.Generator().manual_seed(C * 7 + H + W + shift)
    qkv = torch.randn(2, H, W, 3 * C, generator=g)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    scale = (C // heads) ** -0.5
    ref = _attn_ref(qkv.double(), C, heads, ws, shift, table.double(), mask_kind, scale_after, scale).float()
    exact = _run(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale, torch.float32, False)
    prev = Fn.split_mode()
    Fn.set_split_mode(2)
    try:
        split = _run(qkv, C, heads, ws, shift, table, mask_kind, scale_after, scale, torch.float32, False)
    finally:
        Fn.set_split_mode(prev)
    amax = ref.abs().max().item()
    e_split = (split - ref).abs().max().item()
    e_exact = (exact - ref).abs().max().item()
    assert e_split <= 2e-6 * amax, (e_split, e_exact, amax)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_mfma_attention_strided_views(dtype):
    """qkv and out as channel windows of wider NHWC buffers (ld > 3C, c0 > 0)."""
    import lic_amd.functional as Fn
    C, heads, ws, shift, H, W = 192, 8, 8, 4, 16, 16
    g = torch.Generator().manual_seed(3)
    big = torch.randn(1, H, W, 3 * C + 64, generator=g)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    scale = (C // heads) ** -0.5
    qkv = Fn.Act(big.to(DEV).to(dtype).contiguous(), 32, 3 * C)
    out_buf = torch.full((1, H, W, C + 40), 7.0, device=DEV, dtype=dtype)
    out = Fn.Act(out_buf, 16, C)
    Fn.win_attn(qkv, C, heads, ws, shift, table.to(DEV), heads, 1, 1, False, scale, out=out)
    ref = _attn_ref(big[..., 32:32 + 3 * C].to(dtype).float(), C, heads, ws, shift, table, 1, False, scale)
    got = out_buf[..., 16:16 + C].float().cpu()
    tol = 1e-4 if dtype == torch.float32 else 1e-2 * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= tol
    assert out_buf[..., :16].eq(7).all() and out_buf[..., 16 + C:].eq(7).all()


@pytest.mark.parametrize("C,heads,shift,mask_kind", [(192, 8, 4, 1), (288, 12, 0, 0)])
def test_mfma_attention_8_wave_groups(C, heads, shift, mask_kind):
    """fp16 on >= 1024 windows takes the 8-heads-per-workgroup launch (12 heads: a
    second group with 4 idle waves)."""
    ws, B, H, W = 8, 16, 64, 64
    g = torch.Generator().manual_seed(C + heads)
    qkv = torch.randn(B, H, W, 3 * C, generator=g)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g) * 0.5
    scale = (C // heads) ** -0.5
    ref = _attn_ref(qkv.to(torch.float16).float(), C, heads, ws, shift, table, mask_kind, False, scale)
    out = _run(qkv, C, heads, ws, shift, table, mask_kind, False, scale, torch.float16, False)
    assert (out - ref).abs().max().item() <= 1e-2 * (ref.abs().max().item() + 1e-6)


@pytest.mark.parametrize("B,H,W,shift", [(16, 64, 64, 4), (32, 64, 64, 2), (8, 128, 64, 0), (32, 64, 64, 4),
                                         (2, 64, 64, 4), (1, 16, 16, 4), (1, 32, 64, 0)])
def test_fused_wba_bit_exact(B, H, W, shift):
    """lic_wba_qkv_attn_fwd (csrc/wba_split.hip: fp32x6 qkv Linear + window attention in one launch)
    equals the unfused launches (qkv 1x1 on the virtual-tap split kernel + lic_win_attn_fwd, mfma_mode
    2) bit for bit where the model uses it (>= 64 K pixels: the qkv 1x1 is then a virtual-tap launch),
    and so does WinBasedAttention.run with and without the fusion; on every map the launch matches the
    PyTorch float64 restatement at the fp32x6 bar (smaller maps keep the unfused path, whose qkv runs
    on other split kernels)."""
    from lic_amd import functional as Fn
    from lic_amd.functional import Act
    from lic_amd.layers import win_attention as WA
    torch.manual_seed(7)
    m = WA.WinBasedAttention(dim=192, num_heads=8, window_size=8, shift_size=shift).to(DEV)
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0.0, 0.5)
        m.attn.qkv.bias.normal_(0.0, 0.3)
    x = Act(torch.randn(B, H, W, 192, device=DEV))
    mk = 1 if shift > 0 else 0
    sc = float(m.attn.scale)
    tab = m.attn.relative_position_bias_table
    big = B * H * W >= 65536
    with Fn.split_f32(2):
        assert Fn.wba_qkv_attn_ok(x, 192, 8, 8) == big
        fused = Fn.wba_qkv_attn(x, m.attn.qkv.packed(torch.float32), 8, 8, shift, tab, 8, 1, mk, sc)
        qkv = m.attn.qkv.run(x)
        ref = Fn.win_attn(qkv, 192, 8, 8, shift, tab, 8, 1, mk, False, sc)
        y_fused = m.run(x)
        # the whole block in the one launch (proj + shortcut fused; opt-in LIC_FUSED_WBA_PROJ=1)
        y_proj = Fn.wba_qkv_attn(x, m.attn.qkv.packed(torch.float32), 8, 8, shift, tab, 8, 1, mk, sc,
                                 proj_pk=m.attn.proj.packed(torch.float32))
        y_proj_ref = m.attn.proj.run(fused, r1=x)
        WA._FUSED = False
        try:
            y_ref = m.run(x)
        finally:
            WA._FUSED = True
    torch.cuda.synchronize()
    if big:
        assert torch.equal(fused.t, ref.t)
    assert torch.equal(y_fused.t, y_ref.t)
    if big:   # (smaller maps: the proj 1x1 is not a virtual-tap launch there)
        assert torch.equal(y_proj.t, y_proj_ref.t)
    else:
        assert ((y_proj.t - y_proj_ref.t).abs().max() / y_proj_ref.t.abs().max()).item() < 2e-6
    # and the op itself against float64 torch on the same weights (fp32x6 grade)
    w = m.attn.qkv.weight.detach().double().cpu()
    q64 = x.t.double().cpu() @ w.t() + m.attn.qkv.bias.detach().double().cpu()
    o64 = _attn_ref(q64, 192, 8, 8, shift, tab.detach().double().cpu(), mk, False, sc)
    err = (fused.t.double().cpu() - o64).abs().max() / o64.abs().max()
    assert err < 2e-6, err
