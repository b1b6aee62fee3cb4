"""precision='fp32x6' / 'fp32x3': fp32 activations whose spatial-tile convolutions form every
product from 16-bit parts on the matrix cores (csrc/conv_halo_split.hip; include/lic.h mfma_mode):
fp32x6 = three exact bf16 parts per operand, six products (dropped terms <= 2^-26 relative);
fp32x3 = 2^11 x w ~= x_hi*W1 + x_hi*W2 + x_lo*W1 (x_hi = fp16(x), x_lo = fp16(x - x_hi)), ~3e-7
relative per product (fp32: 6e-8).

Bars: per kernel, max error <= 3e-6 of the output scale against torch fp32 on the CPU and
<= 5e-6 against the exact-fp32 MFMA kernel on the same pack (both sides carry rounding error); end to end, the fp32 parity bars
(bpp 1e-5 against the oracle on the same symbols, tests/parity.check_rate, PSNR 1e-4 dB, symbols by
tests/parity.py, decoder pinned)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R
from parity import check_decoder, check_flip_sets_match, check_rate, check_symbols

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("mode", [2, 1])
@pytest.mark.parametrize("cin,cout,k,s,pad,B,H,epi", [
    (192, 192, 3, 1, (1, 1, 1, 1), 8, 64, "plain"),    # WNSA conv3x3 (16x16 x 192 tiles)
    (192, 192, 7, 1, (3, 3, 3, 3), 8, 64, "lrelu_r1"),  # conv7x7, tap groups
    (192, 192, 5, 2, (1, 1, 2, 2), 8, 128, "plain"),   # ZeroPad2d((1,2,1,2)) + conv5x5 s2 (8x8 x 192 tiles)
    (192, 192, 3, 1, (1, 1, 1, 1), 32, 16, "gelu"),    # slice-loop latents (8x8 x 64 tiles)
    (128, 64, 3, 1, (1, 1, 1, 1), 32, 16, "gate"),     # 8x8 tiles, 64-wide blocks, gate epilogue
    (96, 128, 3, 1, (1, 1, 1, 1), 8, 50, "plain"),     # ragged map, 16x16 x 64 tiles
    (192, 576, 1, 1, (0, 0, 0, 0), 32, 64, "plain"),   # 1x1 qkv Linear of Win_noShift_Attention
    (192, 192, 1, 2, (0, 0, 0, 0), 8, 128, "plain"),   # 1x1 s2 skip of ResidualBlockWithStride (8x8 tiles)
    (192, 192, 1, 1, (0, 0, 0, 0), 8, 128, "square"),  # GDN: conv1x1(x^2) (prologue SQUARE)
    (96, 96, 1, 1, (0, 0, 0, 0), 8, 50, "gate"),       # 1x1 GEMM: ragged M, copad 96 (clamped n-tiles)
    (192, 192, 1, 1, (0, 0, 0, 0), 8, 64, "gdn"),      # 1x1 GEMM: x^2 prologue + GDN x*rsqrt(n) epilogue
    (192, 192, 1, 1, (0, 0, 0, 0), 16, 64, "gdn"),     # 1x1 on the weights-direct kernel's virtual taps
    (96, 96, 1, 1, (0, 0, 0, 0), 32, 60, "gate"),      # virtual taps: ragged tiles, copad 96 < BN 192
    (128, 64, 1, 1, (0, 0, 0, 0), 32, 16, "gelu"),     # slice-loop 1x1 at 16^2: 8x8-px virtual-tap tiles
    (224, 128, 3, 1, (1, 1, 1, 1), 32, 16, "plain"),   # slice-loop cc transform (8x8 px x 64 ch tiles)
    (192, 192, 3, 2, (1, 1, 1, 1), 32, 64, "plain"),   # ResidualBlockWithStride conv3x3 s2: 4/2/2/1-tap phases
    (128, 32, 3, 1, (1, 1, 1, 1), 32, 16, "plain"),    # per-slice 32-channel head (8x8 px x 32 ch tiles)
    (192, 192, 3, 2, (1, 1, 1, 1), 32, 64, "gelu"),    # stride-2 phases, activation on the last phase
    (256, 1152, 3, 1, (1, 1, 1, 1), 32, 8, "plain"),   # h_s 8x8 map: 8x8 px x 64 ch tiles
    (224, 24, 3, 1, (1, 1, 1, 1), 8, 20, "gelu"),      # copad 32 with 8 masked channels, ragged map
    (128, 32, 1, 1, (0, 0, 0, 0), 32, 16, "plain"),    # 32-channel 1x1 on virtual taps
    (192, 192, 7, 1, (3, 3, 3, 3), 32, 16, "gelu"),    # 7x7 on the 16x16 latent: 7 kernel-row launches (8x8 tiles)
    (160, 192, 3, 1, (1, 1, 1, 1), 8, 40, "lrelu_r1"), # 3x3 compile-time addressing (GEO 1), ragged 16x16 tiles
    (192, 192, 5, 2, (1, 1, 2, 2), 32, 32, "gelu"),    # ZeroPad + 5x5 s2 onto 16x16: 9/6/6/4-tap phases, 8x8 tiles
    (64, 64, 3, 1, (1, 1, 1, 1), 32, 4, "lrelu_r1"),   # 4x4 hyper-prior map: one 8x8 tile, 3/4 masked
    (128, 32, 3, 1, (1, 1, 1, 1), 32, 4, "plain"),     # 4x4 map, 32-channel tile
])
def test_split_conv_matches_fp32(cin, cout, k, s, pad, B, H, epi, mode):
    if mode == 1 and (cout % 64 or epi == "gdn" or H < 8):
        pytest.skip("fp32x3 (an extra) keeps the LDS-staged split kernel: 64-channel blocks, maps >= 8, no 1x1 GEMM case")
    import lic_amd.functional as Fn
    from lic_amd import _ffi as L
    from lic_amd.layers import Conv2d
    torch.manual_seed(41 + k + H)
    m = Conv2d(cin, cout, k, s, 0).to(DEV)
    with torch.no_grad():
        m.bias.normal_(0, 0.1)
        if epi == "gdn":     # GDN's norm: gamma >= 0, beta > 0 (model/gdn.py) -> sqrt of a positive sum
            m.weight.abs_()
            m.bias.abs_().add_(0.5)
    x = torch.randn(B, cin, H, H) * 0.5
    X = Fn.Act.from_nchw(x.to(DEV).contiguous(), torch.float32)
    pk = m.packed(torch.float32, pad)
    Ho, Wo = Fn.conv_out_hw(H, H, pk)
    r = Fn.Act.from_nchw(torch.randn(B, cout, Ho, Wo).to(DEV), torch.float32)
    g = Fn.Act.from_nchw(torch.rand(B, cout, Ho, Wo).to(DEV), torch.float32)
    kw = {"plain": {}, "gelu": dict(act=L.ACT_GELU), "lrelu_r1": dict(act=L.ACT_LRELU, r1=r),
          "square": dict(prologue=L.PRO_SQUARE), "abs": dict(prologue=L.PRO_ABS),
          "gdn": dict(prologue=L.PRO_SQUARE, epi=L.EPI_GDN_RSQRT, g=g),
          "gate": dict(act=L.ACT_LRELU, epi=L.EPI_GATE, g=g, r2=r, r1=r)}[epi]
    exact = Fn.conv(X, pk, **kw).nchw().cpu()
    with Fn.split_f32(mode):
        got = Fn.conv(X, pk, **kw).nchw().cpu()
    ws = Fn.split_weights(pk, mode)
    assert ws is not None
    if mode == 2:    # the three bf16 parts sum to the fp32 weights exactly
        assert torch.equal(Fn.split_weights_parts(ws).float().sum(0), pk.w)
    scale = exact.abs().max().item()
    err = (got - exact).abs().max().item()
    base = F.conv2d(F.pad(x, (pad[1], pad[3], pad[0], pad[2])), m.weight.detach().cpu(), m.bias.detach().cpu(), s)
    if epi == "square":
        base = F.conv2d(x * x, m.weight.detach().cpu(), m.bias.detach().cpu(), s)
    if epi == "abs":
        base = F.conv2d(F.pad(x.abs(), (pad[1], pad[3], pad[0], pad[2])), m.weight.detach().cpu(),
                        m.bias.detach().cpu(), s)
    err_cpu = (got - {"plain": base, "gelu": F.gelu(base), "square": base, "abs": base}[epi]).abs().max().item() \
        if epi in ("plain", "gelu", "square", "abs") else 0.0
    print(f"\n[split{mode} conv{k}x{k} {cin}->{cout} B={B} {H}^2 {epi}] max err vs exact-fp32 kernel {err:.2e}, "
          f"vs torch {err_cpu:.2e} (scale {scale:.2f})")
    assert not torch.equal(got, exact)          # the split kernel ran
    assert err <= 5e-6 * scale and err_cpu <= 3e-6 * scale


def _net(arch, B=1, S=256, seed=0, precision="fp32x3"):
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(seed)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    return net_ga.synthetic_syntax_bias_(mod.Net((B, S, S, 3), (B, S, S, 3), False, False, precision=precision), seed)


@pytest.mark.parametrize("precision", ["fp32x6", "fp32x3"])
@pytest.mark.parametrize("arch,B", [("net_ga", 1), ("net_unet_ha_hs", 1), ("net_ga", 32)])
def test_split_net_parity(arch, B, precision):
    """End to end against the oracle, next to the exact-fp32 path on the same weights and input:
    bpp 1e-5 / PSNR 1e-4 dB / decoder pinned, every symbol flip a near-tie (tests/parity.py),
    exactly the exact-fp32 path's set of flipped symbols (positions, not only their count), and
    an RMS error of the latent y no larger than 1.25x the exact path's."""
    net0 = _net(arch, B, precision="fp32")
    P = {k: v.detach().float() for k, v in net0.state_dict().items()}
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(123 + B)) * 2 - 1
    ref = R.net_forward(x, P, arch=arch)
    res = {}
    for prec in ("fp32", precision):
        net = _net(arch, B, precision=prec)
        net.load_state_dict(net0.state_dict())
        net = net.to(DEV)
        bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
        torch.cuda.synchronize()
        flipped = (net.last["symbols"].cpu() != ref["symbols"])
        ne = int(flipped.sum())
        ez = (net.last["z3"].float().cpu() - ref["z3"]).pow(2).mean().sqrt().item()
        res[prec] = (bpp.item(), v_psnr.item(), ne, ez, dict(net.last), flipped)
        del net
    bpp, psnr, flips, ez, last, flipped = res[precision]
    flips0, ez0 = res["fp32"][2], res["fp32"][3]
    print(f"\n[{arch} {precision} B={B}] bpp {bpp:.8f} ref {ref['bpp'].item():.8f} psnr {psnr:.6f} "
          f"ref {ref['v_psnr'].item():.6f} flips {flips} (exact fp32: {flips0}) y rms err {ez:.2e} (exact fp32: {ez0:.2e})")
    check_symbols(last["symbols"], ref, max_rate=max(3e-5, flips0 / ref["symbols"].numel()))
    d = ref["z3"] - ref["means"]
    dist = ((d - torch.floor(d)) - 0.5).abs()
    diff = flipped ^ res["fp32"][5]
    print(f"flip-set difference vs exact fp32: {int(diff.sum())} at |frac-1/2| = {dist[diff].tolist()}; "
          f"all flips: {dist[flipped].tolist()}")
    # the flipped symbols are the exact-fp32 path's, up to oracle ties within 1e-6 of the .5
    # boundary and their cascades (tests/parity.py)
    check_flip_sets_match(flipped, res["fp32"][5], ref)
    assert ez <= 1.25 * ez0
    rate = check_rate(last["likelihoods"], ref, last["symbols"], P, bpp, 65536)
    print(f"rate: d_bpp {rate['d_bpp']:.2e}, on the same symbols {rate['d_bpp_same_symbols']:.2e}, "
          f"flip bits {rate['flip_bits']:.2f}")
    assert abs(psnr - ref["v_psnr"].item()) <= 1e-4
    check_decoder(last, ref, P, flips)


@pytest.mark.parametrize("mode", [2])
@pytest.mark.parametrize("S", [32, 16])
def test_split_conv_transpose_phases(mode, S):
    """s_model's ZeroPad2d((1,0,1,0)) + ConvTranspose2d(5, 2, 3, op=1), 192 -> 192, S^2 -> (2S)^2 at
    B=32: its four sub-pixel phase convolutions (9, 6, 6 and 4 taps) on the weights-direct split
    kernel (16x16-px tiles at S = 32, 8x8-px tiles at S = 16), against torch fp32 on the CPU and the
    exact-fp32 MFMA kernel."""
    import lic_amd.functional as Fn
    from lic_amd.layers import ConvTranspose2d
    torch.manual_seed(61)
    m = ConvTranspose2d(192, 192, 5, 2, 3, output_padding=1).to(DEV)
    with torch.no_grad():
        m.bias.normal_(0, 0.1)
    x = torch.randn(32, 192, S, S) * 0.5
    X = Fn.Act.from_nchw(x.to(DEV).contiguous(), torch.float32)
    exact = m.run(X, prepad=(1, 1)).nchw().cpu()
    with Fn.split_f32(mode):
        got = m.run(X, prepad=(1, 1)).nchw().cpu()
    ref = F.conv_transpose2d(F.pad(x, (1, 0, 1, 0)), m.weight.detach().cpu(), m.bias.detach().cpu(), 2, 3, 1)
    scale = ref.abs().max().item()
    err, err0 = (got - ref).abs().max().item(), (got - exact).abs().max().item()
    print(f"\n[split{mode} convT5x5 s2 B=32 {S}^2] max err vs torch {err:.2e}, vs exact kernel {err0:.2e} (scale {scale:.2f})")
    assert not torch.equal(got, exact)
    assert err <= 3e-6 * scale and err0 <= 5e-6 * scale


@pytest.mark.parametrize("k,s,act", [(3, 2, "lrelu"), (1, 2, "none"), (3, 1, "none")])
def test_split_patch_path_first_conv(k, s, act, monkeypatch):
    """fp32x6: a k x k conv on the 3-channel image runs as a 1x1 conv over its patch map
    (lic_patches, K = 27 -> 32; ResidualBlockWithStride.conv1 / skip at net_ga.py:271); opt-in path."""
    import lic_amd.functional as Fn
    from lic_amd import _ffi as L
    from lic_amd.layers import Conv2d
    import lic_amd.layers._conv as C
    monkeypatch.setattr(C, "_PATCHES", True)
    torch.manual_seed(5 + k + s)
    m = Conv2d(3, 192, k, s, k // 2).to(DEV)
    with torch.no_grad():
        m.bias.normal_(0, 0.1)
    x = torch.rand(8, 3, 64, 64) * 2 - 1
    t = torch.zeros(8, 64, 64, 4, device=DEV)
    t[..., :3] = x.permute(0, 2, 3, 1).to(DEV)
    X = Fn.Act(t, 0, 3, zpad=4)
    kw = dict(act=L.ACT_LRELU) if act == "lrelu" else {}
    exact = m.run(X, **kw).nchw().cpu()
    with Fn.split_f32(2):
        got = m.run(X, **kw).nchw().cpu()
    base = F.conv2d(x.double(), m.weight.detach().cpu().double(), m.bias.detach().cpu().double(), s, k // 2)
    if act == "lrelu":
        base = F.leaky_relu(base, 0.01)
    scale = base.abs().max().item()
    assert got.shape == exact.shape == base.shape
    assert not torch.equal(got, exact)          # the patch path ran (a different summation order)
    assert (got.double() - base).abs().max().item() <= 3e-6 * scale
    assert (got - exact).abs().max().item() <= 5e-6 * scale


@pytest.mark.parametrize("split", [0, 2])
def test_first_conv_one_fp32_chunk_is_bit_identical(split):
    """The image's 3x3 s2 conv (3 channels, zero-padded pixels) packs ONE 8-channel fp32 chunk
    (layers/_conv.py cpad_to=8): bit-identical to the 16-channel pack it replaced (whose second chunk
    was zeros on both sides), on the exact path and with fp32x6 on (it stays on the exact kernel)."""
    import lic_amd.functional as Fn
    from lic_amd import _ffi as L
    from lic_amd.layers import Conv2d
    torch.manual_seed(3)
    m = Conv2d(3, 192, 3, 2, 1).to(DEV)
    with torch.no_grad():
        m.bias.normal_(0, 0.1)
    x = torch.rand(8, 3, 256, 256) * 2 - 1
    X = Fn.Act.from_nchw(x.to(DEV), torch.float32, pad16=True)
    with Fn.split_f32(split):
        got = m.run(X, act=L.ACT_LRELU).nchw().cpu()
        pk16 = m.packed(torch.float32, None, cin_to=4)
        assert pk16.cpad == 16
        ref = Fn.conv(Fn.Act(X.t, X.c0, 4), pk16, act=L.ACT_LRELU).nchw().cpu()
    assert m.packed(torch.float32, None, cin_to=4, cpad_to=8).cpad == 8
    assert torch.equal(got, ref)
    base = F.leaky_relu(F.conv2d(x.double(), m.weight.detach().cpu().double(), m.bias.detach().cpu().double(), 2, 1),
                        0.01)
    assert (got.double() - base).abs().max().item() <= 1e-6 * base.abs().max().item()
