"""BASELINE configs 2 and 3 at their full batch shapes.

The kernels the bench and the sweeps select depend on the batch (conv.hip picks the
32x16-px x 192-ch fp16 tile only when the grid has >= 200 such workgroups, the window
attention goes to 8 waves per workgroup at >= 1024 windows), so the small-batch parity
tests do not cover them.  These run the real shapes and compare every image with the
CPU oracle (oracle/ref_cpu.py, fp32 torch CPU):

  cfg 2: net_ga analysis transform, 32 x 256^2, fp16: y within the fp16 bar (2e-2 of the
         tensor's scale); and the fp32 forward at 32 x 256^2: symbols bit-exact up to
         fp32-summation-order near-ties (tests/parity.py), bpp within 1e-5, PSNR within 1e-4 dB.
  cfg 3: net_unet_ha_hs encode -> quantize -> decode, 16 x 512^2, fp32: same bars, and the
         reconstruction within one uint8 step.
Both forwards run twice: exact fp32 and fp32x6 (the bench headline's precision: fp32
activations and accumulation, six bf16 products of exact three-part splits per product), each
against the same oracle run; the rate bar is tests/parity.check_rate (1e-5 bpp against the oracle
conditioned on the path's own symbols, the measured bits of flipped near-ties reported beside it).
Weights: seeded reference init + net_ga.synthetic_syntax_bias_ (non-degenerate x_rec).
"""
import pytest
import torch

from oracle import ref_cpu as R
from parity import (check_decoder, check_flip_sets_match, check_rate, check_symbols, note_x6_vs_fp32,
                    near_tie_count, record)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(arch, precision, B, S, seed=0):
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(seed)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    return net_ga.synthetic_syntax_bias_(mod.Net((B, S, S, 3), (B, S, S, 3), False, False, precision=precision), seed)


def _x(B, S, seed):
    return torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(seed)) * 2 - 1


def test_cfg2_analysis_b32_fp16():
    from lic_amd.functional import Act
    B, S = 32, 256
    net = _net("net_ga", "fp16", B, S)
    P = {k: v.detach().float() for k, v in net.state_dict().items()}
    net = net.to(DEV)
    x = _x(B, S, 21)
    z3 = net.a_model.run(Act.from_nchw(x.to(DEV), torch.float16, pad16=True)).nchw().float().cpu()
    ref = R.analysis_transform(x, P)
    err = ((z3 - ref).abs().amax(dim=(1, 2, 3)) / ref.abs().amax(dim=(1, 2, 3)))
    print(f"\n[cfg2 a_model fp16 B=32] per-image rel err max {err.max().item():.3e} mean {err.mean().item():.3e}")
    assert err.max().item() < 2e-2


def _check_precision(arch, prec, B, S, net0, x, ref, P):
    """One precision's forward against the oracle: symbols (near-tie rule), rate by
    tests/parity.check_rate (1e-5 bpp against the oracle on the same symbols, batch and per image),
    PSNR 1e-4 dB (batch, and per image on the flip-free images), decoder pinned.  Returns the flip mask."""
    net = _net(arch, prec, B, S)
    net.load_state_dict(net0.state_dict())
    net = net.to(DEV)
    bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
    torch.cuda.synchronize()
    flips = check_symbols(net.last["symbols"], ref)
    flipped = net.last["symbols"].cpu() != ref["symbols"]
    rate = check_rate(net.last["likelihoods"], ref, net.last["symbols"], P, bpp.item(), S * S)
    psnr_img = 20 * torch.log10(255 / torch.sqrt(v_mse.double().cpu()))
    psnr_img_ref = 20 * torch.log10(255 / torch.sqrt(ref["v_mse"].double()))
    # per-image PSNR vs the free-running oracle on the images without a flipped symbol; an image with
    # one decodes another y_hat there and is pinned on its own y_hat by check_decoder
    clean = ~flipped.flatten(1).any(1)
    d_img = (psnr_img - psnr_img_ref).abs()[clean]
    print(f"\n[{arch} {prec} B={B} {S}^2] flips {flips} d_bpp {rate['d_bpp']:.2e} (same symbols "
          f"{rate['d_bpp_same_symbols']:.2e}, per image max {rate['d_bpp_per_image']:.2e}; flip bits "
          f"{rate['flip_bits']:.2f}) d_psnr {abs(v_psnr.item() - ref['v_psnr'].item()):.2e} "
          f"(per flip-free image max {d_img.max().item() if d_img.numel() else 0.0:.2e}, {int(clean.sum())} images)")
    record(f"{arch} B={B} {S}x{S}", prec, flips=flips, near_ties=near_tie_count(net.last["symbols"], ref),
           d_bpp=rate["d_bpp"], d_bpp_same_symbols=rate["d_bpp_same_symbols"], flip_bits=rate["flip_bits"],
           d_psnr_db=abs(v_psnr.item() - ref["v_psnr"].item()), symbols=int(ref["symbols"].numel()))
    assert abs(v_psnr.item() - ref["v_psnr"].item()) <= 1e-4
    assert d_img.numel() == 0 or d_img.max().item() <= 1e-4
    check_decoder(net.last, ref, P, flips)
    del net
    torch.cuda.empty_cache()
    return flipped, rate["d_bpp"]


def _compare_forward(arch, B, S, seed, xseed, precisions=("fp32", "fp32x6")):
    """The exact-fp32 path and the headline's fp32x6 path on the same weights and batch, against
    one oracle run; the two fp32-grade paths flip the same symbols up to oracle ties within 1e-6
    of the .5 boundary and their cascades (tests/parity.check_flip_sets_match)."""
    net0 = _net(arch, "fp32", B, S, seed)
    P = {k: v.detach().float() for k, v in net0.state_dict().items()}
    x = _x(B, S, xseed)
    ref = R.net_forward(x, P, arch=arch)
    res = {p: _check_precision(arch, p, B, S, net0, x, ref, P) for p in precisions}
    masks = {p: r[0] for p, r in res.items()}
    if "fp32" in masks and "fp32x6" in masks:
        n = check_flip_sets_match(masks["fp32x6"], masks["fp32"], ref)
        print(f"flip-set difference fp32x6 vs exact fp32: {n}")
    note_x6_vs_fp32({p: r[1] for p, r in res.items()})


def test_cfg2_forward_b32_fp32_bit_exact_symbols():
    _compare_forward("net_ga", 32, 256, 0, 22)


def test_cfg3_net_unet_ha_hs_b16_512_fp32():
    _compare_forward("net_unet_ha_hs", 16, 512, 0, 23)


@pytest.mark.timeout(900)
def test_cfg2_gate_panel():
    """The headline precision's parity over a panel of config-2 batches (net_ga, B=32, 256^2, seed-0 weights;
    input seeds 1000 = the bench's timed batch, 22 = the batch above, 1..8), bench.py's precision gate run as a
    test: on every batch each fp32x6 flip is an oracle near-tie or its cascade, the same-symbol rate is within
    1e-5 bpp and the PSNR within 1e-4 dB; over the panel fp32x6 flips no more symbols than exact fp32 and its
    worst free-running delta-bpp is no worse than max(1e-5, exact fp32's) (the committed
    panel: profiles/r06/parity_panel_cfg2.jsonl)."""
    import bench
    ok, panel, _, _ = bench.gate_panel("net_ga", 256, torch.device(DEV), 32)
    print(f"\n[cfg2 panel] total flips {panel['total_flips']} worst d_bpp {panel['worst_d_bpp']} "
          f"batches meeting the bar {panel['batches_meeting_bar']}")
    record("net_ga B=32 256x256 panel", "fp32x6 vs fp32", total_flips=panel["total_flips"],
           worst_d_bpp=panel["worst_d_bpp"], seeds=panel["seeds"])
    assert panel["fp32x6_every_batch_ties_and_same_symbol_rate_ok"], panel["rows"]["fp32x6"]
    assert ok, panel
