"""Known-answer tests pinning the CPU oracle (oracle/ref_cpu.py).  The reference
ships no tests, fixtures or checkpoints and cannot be run here,
so these analytic identities are the oracle's pin."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R


def _gdn_params(C, pfx, gamma_scale=0.1, seed=0, compressai=False):
    g = torch.Generator().manual_seed(seed)
    P = {}
    ped = torch.Tensor([(2 ** -18) ** 2])
    if compressai:
        P[pfx + ".beta"] = R.nnp_init(torch.ones(C) + 0.5 * torch.rand(C, generator=g), ped)
        P[pfx + ".gamma"] = R.nnp_init(gamma_scale * torch.eye(C) + 0.01 * torch.rand(C, C, generator=g), ped)
        P[pfx + ".beta_reparam.pedestal"] = ped
        P[pfx + ".gamma_reparam.pedestal"] = ped
        P[pfx + ".beta_reparam.lower_bound.bound"] = torch.Tensor([(1e-6 + (2 ** -18) ** 2) ** 0.5])
        P[pfx + ".gamma_reparam.lower_bound.bound"] = torch.Tensor([(0 + (2 ** -18) ** 2) ** 0.5])
    else:
        ro = torch.FloatTensor([2 ** -18])
        P[pfx + ".reparam_offset"] = ro
        P[pfx + ".pedestal"] = ro ** 2
        P[pfx + ".beta"] = torch.sqrt(torch.ones(C) + 0.5 * torch.rand(C, generator=g) + ro ** 2)
        P[pfx + ".gamma"] = torch.sqrt(gamma_scale * torch.eye(C) + 0.01 * torch.rand(C, C, generator=g) + ro ** 2)
    return P


def test_nnp_roundtrip():
    """ops/parametrizers.py:52-58: init -> forward returns 0.1*I."""
    ped = torch.Tensor([(2 ** -18) ** 2])
    bound = torch.Tensor([(0 + (2 ** -18) ** 2) ** 0.5])
    g = R.nnp_init(0.1 * torch.eye(5), ped)
    out = R.nnp_forward(g, bound, ped)
    torch.testing.assert_close(out, 0.1 * torch.eye(5), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("variant", ["model", "compressai"])
def test_gdn_gamma_zero(variant):
    """GDN with Gamma' = 0 returns x / sqrt(beta')."""
    C = 6
    x = torch.randn(2, C, 5, 5)
    P = _gdn_params(C, "g", compressai=variant == "compressai")
    P["g.gamma"] = torch.zeros(C, C)  # clamps to the lower bound -> gamma' = bound^2 - pedestal ~ 0
    if variant == "compressai":
        beta = R.nnp_forward(P["g.beta"], P["g.beta_reparam.lower_bound.bound"], P["g.beta_reparam.pedestal"])
        out = R.gdn_compressai(x, P, "g")
    else:
        ped, bb, gb = R.gdn_model_bounds(P, "g")
        beta = torch.max(P["g.beta"], bb) ** 2 - ped
        out = R.gdn_model(x, P, "g")
    ref = x / torch.sqrt(beta).view(1, C, 1, 1)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)


def test_igdn_is_x_times_sqrt_norm():
    C = 4
    x = torch.randn(1, C, 3, 3)
    P = _gdn_params(C, "g")
    ped, bb, gb = R.gdn_model_bounds(P, "g")
    beta = torch.max(P["g.beta"], bb) ** 2 - ped
    gamma = torch.max(P["g.gamma"], gb) ** 2 - ped
    norm = torch.einsum("oi,bihw->bohw", gamma, x ** 2) + beta.view(1, C, 1, 1)
    torch.testing.assert_close(R.gdn_model(x, P, "g", inverse=True), x * torch.sqrt(norm), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(R.gdn_model(x, P, "g"), x / torch.sqrt(norm), rtol=1e-5, atol=1e-6)


def _wba_params(C, heads, ws, pfx, zero=False, seed=0):
    g = torch.Generator().manual_seed(seed)
    mk = (lambda *s: torch.zeros(*s)) if zero else (lambda *s: 0.2 * torch.randn(*s, generator=g))
    return {pfx + ".attn.relative_position_bias_table": mk((2 * ws - 1) ** 2, heads),
            pfx + ".attn.qkv.weight": mk(3 * C, C), pfx + ".attn.qkv.bias": mk(3 * C),
            pfx + ".attn.proj.weight": mk(C, C), pfx + ".attn.proj.bias": mk(C)}


def test_wba_zero_weights_is_identity():
    x = torch.randn(2, 16, 8, 8)
    P = _wba_params(16, 4, 4, "w", zero=True)
    torch.testing.assert_close(R.win_based_attention(x, P, "w", 4, 4, 2), x)


def test_window_partition_bijection():
    x = torch.randn(2, 16, 8, 3)
    w = R.window_partition(x, 4)
    assert w.shape == (2 * 4 * 2, 4, 4, 3)
    torch.testing.assert_close(R.window_reverse(w, 4, 16, 8), x)


def test_wba_mask_full_window_when_ws_equals_h():
    """With ws == H == W a single window holds all tokens; regions split at H - shift."""
    m = R.wba_mask(4, 4, 4, 2)
    assert m.shape == (1, 16, 16)
    lab = torch.tensor([[0 if y < 2 else 1 for y in range(4)]]).T * 3 + torch.tensor([[0 if x < 2 else 1 for x in range(4)]])
    lab = lab.reshape(-1)
    expect = torch.where(lab[None, :] != lab[:, None], -100.0, 0.0)
    torch.testing.assert_close(m[0], expect)


def test_wba_equivariant_to_window_permutation_without_shift():
    """Without shift, attention is per-window: permuting whole windows commutes with WBA."""
    torch.manual_seed(0)
    x = torch.randn(1, 8, 8, 8)
    P = _wba_params(8, 2, 4, "w")
    y = R.win_based_attention(x, P, "w", 2, 4, 0)
    xs = torch.cat([x[:, :, 4:], x[:, :, :4]], dim=2)
    ys = R.win_based_attention(xs, P, "w", 2, 4, 0)
    torch.testing.assert_close(torch.cat([ys[:, :, 4:], ys[:, :, :4]], 2), y, rtol=1e-5, atol=1e-6)


def test_gaussian_likelihood_integrates_to_one():
    """Sum over integer bins of the unit-bin likelihood is 1 (means/scale fixed)."""
    mu, s = torch.tensor([0.3]), torch.tensor([1.7])
    k = torch.arange(-60, 61, dtype=torch.float32)
    L = R.gaussian_likelihood(k + 0.0 * mu, s.expand_as(k), mu.expand_as(k))
    assert abs(L.sum().item() - 1.0) < 1e-5
    assert torch.all(L >= 1e-9)


def test_likelihood_scale_bound_and_floor():
    L = R.gaussian_likelihood(torch.tensor([0.0, 40.0]), torch.tensor([1e-3, 1e-3]), torch.tensor([0.0, 0.0]))
    # scale clamps to 0.11: P(|v|<=0.5) at s=0.11 is ~1; far tail clamps to 1e-9
    assert abs(L[0].item() - (1 - math.erfc(0.5 / 0.11 / math.sqrt(2)))) < 1e-6
    assert abs(L[1].item() - 1e-9) < 1e-15


def test_round_half_even():
    y = torch.tensor([0.5, 1.5, 2.5, -0.5, -1.5, 2.4999999])
    assert R.symbols(y, torch.zeros_like(y)).tolist() == [0, 2, 2, 0, -2, 2]


def test_ste_round_forward_is_round():
    x = torch.randn(10000) * 10
    assert torch.equal(R.ste_round(x), torch.round(x))


def test_batch_conv_is_per_image_1x1():
    torch.manual_seed(0)
    w = torch.randn(3, 3, 16, 1, 1)
    x = torch.randn(3, 16, 5, 5)
    out = R.batch_conv(w, x)
    ref = torch.einsum("boc,bchw->bohw", w[..., 0, 0], x)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_han_lam_csam_identity_at_zero_gamma_and_lam_known_answer():
    """han.py LAM / CSAM with gamma = 0 are identities (default init); LAM on two
    orthogonal unit maps: energy = I, energy_new = 1 - I, softmax rows = [1, e] / (1 + e)."""
    import math
    x = torch.randn(2, 5, 4, 3, 3)
    assert torch.equal(R.han_lam(x, torch.zeros(1)), x.view(2, 20, 3, 3))
    P = {"c.conv.weight": torch.randn(1, 1, 3, 3, 3), "c.conv.bias": torch.randn(1), "c.gamma": torch.zeros(1)}
    y = torch.randn(1, 4, 5, 5)
    assert torch.equal(R.han_csam(y, P, "c"), y)
    e0 = torch.zeros(1, 2, 1, 1, 2)
    e0[0, 0, 0, 0, 0] = 1.0
    e0[0, 1, 0, 0, 1] = 1.0
    out = R.han_lam(e0, torch.ones(1)).view(1, 2, 1, 1, 2)
    a_self, a_other = 1 / (1 + math.e), math.e / (1 + math.e)
    torch.testing.assert_close(out[0, 0, 0, 0], torch.tensor([1 + a_self, a_other]))


def test_parity_check_symbols_accepts_only_near_ties():
    """tests/parity.check_symbols: a flip at a near-.5 tie of the oracle's y - mu passes, a flip
    anywhere else fails."""
    import pytest as _pt
    from parity import check_symbols
    g = torch.Generator().manual_seed(0)
    z3 = torch.randn(1, 8, 16, 16, generator=g) * 3
    mu = torch.randn(1, 8, 16, 16, generator=g)
    z3[0, 5, 3, 3] = mu[0, 5, 3, 3] + 2.5 + 1e-5           # near-tie
    ref = {"z3": z3, "means": mu, "symbols": torch.round(z3 - mu).to(torch.int32)}
    sym = ref["symbols"].clone()
    assert check_symbols(sym, ref) == 0
    sym[0, 5, 3, 3] += 1
    assert check_symbols(sym, ref, max_rate=1e-2) == 1
    sym[0, 1, 12, 12] += 1                                   # no tie, no earlier flip nearby
    with _pt.raises(AssertionError):
        check_symbols(sym, ref, max_rate=1e-2)


def test_counter_noise_is_uniform_and_seeded():
    u = R.counter_noise(3, (2, 8, 8, 48))
    assert u.shape == (2, 8, 8, 48) and u.min() >= -0.5 and u.max() < 0.5
    assert abs(u.mean().item()) < 0.02 and abs(u.var().item() - 1 / 12) < 0.01
    assert torch.equal(u, R.counter_noise(3, (2, 8, 8, 48)))
    assert not torch.equal(u, R.counter_noise(4, (2, 8, 8, 48)))


def test_slice_loop_forced_symbols():
    """oracle.slice_loop(forced_symbols=...): forcing the oracle's own symbols reproduces its
    likelihoods bitwise; forcing one flipped symbol of slice 0 changes that symbol's likelihood
    and the contexts (mu / sigma) of later slices only, never an earlier or the same slice's
    other symbols (tests/parity.check_rate conditions the oracle on a GPU path's symbols)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden as MG
    P = MG.state_of(MG.make_net("net_ga", 256, 0))
    x = MG.seeded_image(1, 256, 3)
    ref = R.net_forward(x, P, arch="net_ga")
    args = (ref["z3"], ref["latent_means"], ref["latent_scales"], P)
    _, lik, sym, mu, sc = R.slice_loop(*args, forced_symbols=ref["symbols"].to(torch.int32))
    assert torch.equal(lik, ref["likelihoods"]) and torch.equal(mu, ref["means"]) and torch.equal(sc, ref["scales"])
    forced = ref["symbols"].to(torch.int32).clone()
    forced[0, 5, 1, 2] += 1
    _, lik2, sym2, mu2, sc2 = R.slice_loop(*args, forced_symbols=forced)
    assert torch.equal(sym2, forced)
    changed = lik2 != lik
    assert changed[0, 5, 1, 2]
    assert not changed[:, :48].flatten()[torch.arange(48 * 256) != (5 * 256 + 1 * 16 + 2)].any()
    assert torch.equal(mu2[:, :48], mu[:, :48]) and not torch.equal(mu2[:, 48:], mu[:, 48:])
