"""End-to-end parity of Net.forward(x, 'test') on the HIP path against the CPU
oracle (oracle/ref_cpu.net_forward) with the same state_dict and seeded input.

Bar (BASELINE.json north_star): bpp within 1e-5, PSNR within 1e-4 dB, symbol indices
bit-exact (0 flipped symbols on the fp32 path), and the decoder side pinned directly:
the syntax vector before rounding, x_tilde = s_model(y_hat) and the uint8 reconstruction.
Weights are the seeded reference init + net_ga.synthetic_syntax_bias_ (otherwise the
rounded syntax is 0 and x_rec does not depend on s_model)."""
import math

import pytest
import torch

from oracle import ref_cpu as R
from parity import (check_decoder, check_flip_sets_match, check_rate, check_symbols, note_x6_vs_fp32,
                    near_tie_count, record)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _make(arch, precision, seed=0, size=256):
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.manual_seed(seed)
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    net = mod.Net((1, size, size, 3), (1, size, size, 3), False, False, precision=precision)
    return net_ga.synthetic_syntax_bias_(net, seed)


def _input(B, size, seed=123):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, 3, size, size, generator=g) * 2 - 1


@pytest.mark.parametrize("arch", ["net_ga", "net_unet_ha_hs"])
def test_net_fp32_parity(arch):
    net = _make(arch, "fp32")
    P = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    net = net.to(DEV)
    x = _input(1, 256)
    bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
    torch.cuda.synchronize()
    ref = R.net_forward(x, P, arch=arch)
    z3 = net.last["z3"].float().cpu()
    rel = ((z3 - ref["z3"]).abs().max() / ref["z3"].abs().max()).item()
    assert rel < 1e-4, rel
    sym = net.last["symbols"].cpu()
    mism = (sym != ref["symbols"]).float().mean().item()
    print(f"\n[{arch} fp32] bpp gpu={bpp.item():.8f} ref={ref['bpp'].item():.8f} "
          f"psnr gpu={v_psnr.item():.6f} ref={ref['v_psnr'].item():.6f} z3 rel={rel:.2e} sym mismatch={mism:.2e}")
    assert mism == 0
    check_decoder(net.last, ref, P, 0)
    assert abs(bpp.item() - ref["bpp"].item()) <= 1e-5 * max(1.0, abs(ref["bpp"].item()))
    assert abs(v_psnr.item() - ref["v_psnr"].item()) <= 1e-4 or math.isinf(ref["v_psnr"].item())


@pytest.mark.parametrize("arch", ["net_ga"])
def test_net_fp16_close(arch):
    net = _make(arch, "fp16")
    P = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    net = net.to(DEV)
    x = _input(1, 256)
    bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
    ref = R.net_forward(x, P, arch=arch)
    z3 = net.last["z3"].float().cpu()
    rel = ((z3 - ref["z3"]).abs().max() / ref["z3"].abs().max()).item()
    sym = net.last["symbols"].cpu()
    mism = (sym != ref["symbols"]).float().mean().item()
    print(f"\n[{arch} fp16] bpp gpu={bpp.item():.6f} ref={ref['bpp'].item():.6f} "
          f"psnr gpu={v_psnr.item():.4f} ref={ref['v_psnr'].item():.4f} z3 rel={rel:.2e} sym mismatch={mism:.2e}")
    assert rel < 5e-2
    assert abs(bpp.item() - ref["bpp"].item()) <= 2e-2 * max(1.0, abs(ref["bpp"].item()))


def test_net_deterministic():
    net = _make("net_ga", "fp32").to(DEV)
    x = _input(2, 256).to(DEV)
    a = net(x, "test", return_intermediates=True)
    s1 = net.last["symbols"].clone()
    b = net(x, "test", return_intermediates=True)
    assert torch.equal(s1, net.last["symbols"])
    assert a[0].item() == b[0].item() and a[2].item() == b[2].item()


@pytest.mark.parametrize("arch,hw", [("net_ga", (768, 512)), ("net_unet_ha_hs", (512, 768))])
def test_net_fp32_parity_kodak_shape(arch, hw):
    """BASELINE config 4 shapes (Kodak 768x512 landscape / 512x768 portrait, H != W): the
    synthetic Kodak stand-in of eval_net.py against the oracle, on the exact-fp32 path and on
    the headline's fp32x6 path (the tile choice depends on the map size), one oracle run."""
    import eval_net
    from lic_amd.model import net_ga, net_unet_ha_hs
    H, W = hw
    mod = net_ga if arch == "net_ga" else net_unet_ha_hs
    x = eval_net.synthetic_image(4, H, W).unsqueeze(0) * 2 - 1
    ref, P, masks, d_bpp = None, None, {}, {}
    for prec in ("fp32", "fp32x6"):
        torch.manual_seed(2)
        net = net_ga.synthetic_syntax_bias_(mod.Net((1, H, W, 3), (1, H, W, 3), False, False, precision=prec), 2)
        if ref is None:
            sd = net.state_dict()
            P = {k: v.detach().float().cpu() for k, v in sd.items()}
            ref = R.net_forward(x, P, arch=arch)
        else:
            net.load_state_dict(sd)
        net = net.to(DEV)
        bpp, v_mse, v_psnr = net(x.to(DEV), "test", return_intermediates=True)
        torch.cuda.synchronize()
        # 294,912 symbols: fp32 summation order may flip the odd near-tie (tests/parity.py); the
        # 1e-5 bpp bar binds against the oracle on the same symbols, the flips' measured bits are reported
        flips = check_symbols(net.last["symbols"], ref)
        masks[prec] = net.last["symbols"].cpu() != ref["symbols"]
        rate = check_rate(net.last["likelihoods"], ref, net.last["symbols"], P, bpp.item(), H * W)
        print(f"\n[{arch} {H}x{W} {prec}] bpp gpu={bpp.item():.8f} ref={ref['bpp'].item():.8f} "
              f"psnr gpu={v_psnr.item():.6f} ref={ref['v_psnr'].item():.6f} flips {flips} "
              f"(d_bpp on the same symbols {rate['d_bpp_same_symbols']:.2e}, flip bits {rate['flip_bits']:.2f})")
        record(f"{arch} B=1 {H}x{W} (config 4 shape)", prec, flips=flips,
               near_ties=near_tie_count(net.last["symbols"], ref), d_bpp=rate["d_bpp"],
               d_bpp_same_symbols=rate["d_bpp_same_symbols"], flip_bits=rate["flip_bits"],
               d_psnr_db=abs(v_psnr.item() - ref["v_psnr"].item()), symbols=int(ref["symbols"].numel()))
        d_bpp[prec] = rate["d_bpp"]
        assert abs(v_psnr.item() - ref["v_psnr"].item()) <= 1e-4
        check_decoder(net.last, ref, P, flips)
        del net
    check_flip_sets_match(masks["fp32x6"], masks["fp32"], ref)
    note_x6_vs_fp32(d_bpp)


def test_rd_sweep_runs_two_lambdas():
    """eval_net --synthetic-kodak: the config-4 sweep (2 lambdas, graph replay) on one GPU, batched per
    image shape (the default) and one image per forward: the same per-image means."""
    import eval_net
    res = {}
    for batched in (True, False):
        summ, ips, world = eval_net.rd_sweep([0.0018, 0.0932], "", arch="net_ga", precision="fp32x6", graph=True,
                                             batched=batched)
        assert world == 1 and len(summ) == 2 and all(s["images"] == 24 for s in summ)
        assert all(math.isfinite(s["bpp"]) and s["bpp"] > 0 and math.isfinite(s["psnr"]) for s in summ)
        assert ips > 0
        res[batched] = summ
        print(f"\n[rd sweep fp32x6 {'batched' if batched else 'per image'}] {ips:.1f} images/s; " +
              "; ".join(f"{s['lambda']}: {s['bpp']:.6f} bpp {s['psnr']:.5f} dB" for s in summ))
    for a, b in zip(res[True], res[False]):
        # per-image means of the same images; only fp32 summation order differs (batch-size-dependent
        # tiles): the bar is the north-star one
        assert abs(a["bpp"] - b["bpp"]) <= 1e-5 and abs(a["psnr"] - b["psnr"]) <= 1e-4, (a, b)


@pytest.mark.parametrize("arch", ["net_ga", "net_unet_ha_hs"])
def test_seeded_noise_eval_mode(arch):
    """The reference's eval bpp is stochastic (its nets stay in training mode, so
    GaussianConditional prices y + U(-1/2, 1/2): net_ga.py:1049, eval_net.py:90-96).
    Net.forward(x, 'test', noise_seed=s) reproduces that mode with a seeded stream: bpp vs the
    oracle with the same stream (1e-5), symbols / PSNR unchanged, another seed another bpp,
    and the same seed in mode 'train' prices the same noisy values."""
    net = _make(arch, "fp32")
    P = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    net = net.to(DEV)
    x = _input(1, 256, seed=31)
    bpp0, _, psnr0 = net(x.to(DEV), "test")
    bpp1, _, psnr1 = net(x.to(DEV), "test", return_intermediates=True, noise_seed=7)
    sym1 = net.last["symbols"].cpu()
    bpp2, _, _ = net(x.to(DEV), "test", noise_seed=8)
    ref = R.net_forward(x, P, arch=arch, noise_seed=7)
    print(f"\n[{arch} noise eval] bpp dequantize {bpp0.item():.6f} seed7 {bpp1.item():.6f} (ref {ref['bpp'].item():.6f}) "
          f"seed8 {bpp2.item():.6f}")
    assert abs(bpp1.item() - ref["bpp"].item()) <= 1e-5 * max(1.0, abs(ref["bpp"].item()))
    assert check_symbols(sym1, ref) == 0
    assert psnr1.item() == psnr0.item()
    assert bpp1.item() != bpp0.item() and bpp2.item() != bpp1.item()
    if arch == "net_ga":
        with torch.no_grad():
            bpp_t, _ = net(x.to(DEV), "train", seed=7)
        assert abs(bpp_t.item() - bpp1.item()) <= 1e-4 * abs(bpp1.item())
