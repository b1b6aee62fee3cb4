"""Generate the committed golden fixtures under tests/golden/ (test infrastructure).

The reference ships no tests, fixtures or checkpoints and cannot be run here
(SURVEY.md 8(c) records a binding permission denial), so these vectors are produced
by the CPU oracle (oracle/ref_cpu.py) on seeded inputs and seeded reference-init
weights.  They freeze the oracle's outputs so that (1) a change to the oracle is
caught by the CPU suite (tests/test_golden.py, `not gpu`) and (2) the HIP path is
checked against fixed vectors on the GPU box without recomputing the oracle.
Parity status of the oracle itself: unpinned (see oracle/ref_cpu.py header).

Files (numpy .npz, no pickles):
  ops.npz           per-op vectors: GDN / IGDN (model/gdn.py and compressai variants),
                    WinBasedAttention (layers/win_attention.py:119-209), Gaussian
                    likelihood + symbols incl. forced .5 ties (compressai
                    GaussianConditional, net_ga.py:1049), ste_round ties.
  net_ga_256.npz    Net.forward(x,'test') of model/net_ga.py, 1x3x256x256, fp32.
  net_unet_ha_hs_256.npz  same for model/net_unet_ha_hs.py.
  source_net_256.npz      source_net z (BASELINE config 1), 1x3x256x256.
Network weights are not stored (67 M parameters): they are re-created by
torch.manual_seed(seed) + the reference's init (weight_init, net_ga.py:723-729) +
lic_amd.model.net_ga.synthetic_syntax_bias_ (Syntax_Model.conv bias offset so that the
rounded syntax and hence the reconstruction are not identically zero);
`param_sum` / `param_abs_sum` pin that the regenerated weights are identical.
The net fixtures hold the syntax vector before rounding, x_tilde (every 8th pixel),
x_rec as uint8 (non-constant: asserted) and the per-slice symbols / bpp / PSNR.

usage: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import lic_amd  # noqa: E402,F401
from oracle import ref_cpu as R  # noqa: E402

NET_SEED = 0
X_SEED = 5
SIZE = 256


def seeded_image(B, size, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, 3, size, size, generator=g) * 2 - 1


def make_net(arch, size=SIZE, seed=NET_SEED):
    from lic_amd.model import net_ga, net_unet_ha_hs, source_net
    torch.manual_seed(seed)
    mod = {"net_ga": net_ga, "net_unet_ha_hs": net_unet_ha_hs, "source_net": source_net}[arch]
    net = mod.Net((1, size, size, 3), (1, size, size, 3), False, False, precision="fp32")
    if arch != "source_net":
        net_ga.synthetic_syntax_bias_(net, seed)
    return net


def x_rec_u8(x_rec):
    """x_hat of net_ga.py:1137 as uint8."""
    return torch.round(torch.clamp((x_rec + 1) * 127.5, 0, 255)).to(torch.uint8)


def state_of(net):
    return {k: v.detach().float().cpu() for k, v in net.state_dict().items()}


def param_sums(P):
    s = sum(float(v.double().sum()) for v in P.values())
    a = sum(float(v.double().abs().sum()) for v in P.values())
    return np.float64(s), np.float64(a)


def op_modules():
    """Seeded per-op modules (shared by the generator and tests/test_golden.py)."""
    from lic_amd.layers import GDN as CGDN, WinBasedAttention
    from lic_amd.model.gdn import GDN, IGDN
    torch.manual_seed(21)
    C = 16
    mods = {"gdn_model": GDN(C), "igdn_model": IGDN(C, inverse=True), "gdn_compressai": CGDN(C)}
    with torch.no_grad():
        for m in mods.values():
            m.beta.add_(0.3 * torch.rand(C))
            m.gamma.add_(0.05 * torch.rand(C, C))
    wba = WinBasedAttention(32, 8, 4, 2)
    with torch.no_grad():
        for p in wba.parameters():
            p.normal_(0, 0.05)
    mods["wba"] = wba
    return mods


def make_ops():
    out = {}
    mods = op_modules()
    g = torch.Generator().manual_seed(22)
    x = torch.randn(2, 16, 5, 6, generator=g) * 2
    out["gdn.x"] = x
    for name in ("gdn_model", "igdn_model", "gdn_compressai"):
        P = {"g." + k: v.detach().float() for k, v in mods[name].state_dict().items()}
        if name == "gdn_compressai":
            ref = R.gdn_compressai(x, P, "g")
        else:
            ref = R.gdn_model(x, P, "g", inverse=(name == "igdn_model"))
        out[name + ".y"] = ref
    xw = torch.randn(2, 32, 8, 8, generator=g)
    P = {"w." + k: v.detach().float() for k, v in mods["wba"].state_dict().items()}
    out["wba.x"] = xw
    out["wba.y"] = R.win_based_attention(xw, P, "w", 8, 4, 2)
    # Gaussian rate: half of the entries sit exactly on .5 ties of (y - mu)
    y = torch.randn(2, 8, 6, 6, generator=g) * 4
    mu = torch.randn(2, 8, 6, 6, generator=g)
    sigma = torch.rand(2, 8, 6, 6, generator=g) * 3
    tie = torch.rand(2, 8, 6, 6, generator=g) < 0.5
    k = torch.randint(-6, 6, (2, 8, 6, 6), generator=g).float()
    mu = torch.where(tie, torch.round(mu * 4) / 4, mu)  # exactly representable mu
    y = torch.where(tie, mu + k + 0.5, y)
    out["rate.y"], out["rate.mu"], out["rate.sigma"] = y, mu, sigma
    out["rate.symbols"] = R.symbols(y, mu)
    out["rate.yhat"] = R.quantize_dequantize(y, mu)
    # compressai GaussianConditional.forward prices the quantized outputs (net_ga.py:1049)
    out["rate.likelihood"] = R.gaussian_likelihood(out["rate.yhat"], sigma, mu)
    t = torch.tensor([-2.5, -1.5, -0.5, 0.5, 1.5, 2.5, 0.49999997, -0.49999997])
    out["ste.x"], out["ste.y"] = t, R.ste_round(t)
    np.savez(os.path.join(HERE, "ops.npz"), **{k: v.numpy() for k, v in out.items()})


def make_net_fixture(arch):
    net = make_net(arch)
    P = state_of(net)
    x = seeded_image(1, SIZE, X_SEED)
    s, a = param_sums(P)
    if arch == "source_net":
        z = R.source_net_forward(x, P)
        np.savez(os.path.join(HERE, f"{arch}_{SIZE}.npz"), net_seed=NET_SEED, x_seed=X_SEED, size=SIZE,
                 param_sum=s, param_abs_sum=a, z=z.numpy())
        return
    r = R.net_forward(x, P, arch=arch)
    sym = r["symbols"]
    assert sym.abs().max() < 2 ** 15
    u8 = x_rec_u8(r["x_rec"])
    assert u8.unique().numel() > 1, "degenerate reconstruction (syntax rounds to 0)"
    assert torch.round(r["syntax"]).abs().sum() > 0
    np.savez_compressed(os.path.join(HERE, f"{arch}_{SIZE}.npz"), net_seed=NET_SEED, x_seed=X_SEED, size=SIZE,
                        param_sum=s, param_abs_sum=a, bpp=r["bpp"].numpy(), v_psnr=r["v_psnr"].numpy(),
                        v_mse=r["v_mse"].numpy(), symbols=sym.to(torch.int16).numpy(), z_hat=r["z_hat"].numpy(),
                        syntax=r["syntax"].numpy(), x_tilde_s8=r["x_tilde"][:, :, ::8, ::8].contiguous().numpy(),
                        x_rec_u8=u8.numpy())


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    make_ops()
    for arch in ("net_ga", "net_unet_ha_hs", "source_net"):
        make_net_fixture(arch)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")
