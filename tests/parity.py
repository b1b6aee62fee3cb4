"""Shared end-to-end parity checks of the quantised symbols against the CPU oracle.

The symbols are bit-exact given identical (y, mu) (tests/test_gpu_ops.py, ties to even
included).  End to end, y and mu come from ~10^8 fp32 multiply-adds whose summation order
differs between MFMA tiles and oneDNN, so they differ from the oracle's by ~1e-6 relative,
and a symbol whose reference value y - mu lies within that distance of a .5 rounding
boundary can round the other way (the oracle's own value is as far from the exact one).
``check_symbols`` therefore requires every mismatch to be such a near-tie of the oracle's
y - mu (or to sit next to an earlier near-tie flip: a flipped y_hat of slice i moves mu of
the later slices in its window), and bounds the rate; with no near-ties the result is
bit-exact (all 256^2 cases measure 0 flips).
"""
import torch

TIE_EPS = 2e-4      # |frac(y - mu) - 0.5| of a summation-order flip (measured <= 1e-4)


def check_symbols(sym_gpu: torch.Tensor, ref: dict, max_rate: float = 3e-5) -> int:
    sym_gpu = sym_gpu.cpu()
    ne = sym_gpu != ref["symbols"]
    n = int(ne.sum())
    if n == 0:
        return 0
    d = (ref["z3"] - ref["means"])
    dist = ((d - torch.floor(d)) - 0.5).abs()
    near_tie = ne & (dist < TIE_EPS)
    # cascades: a non-tie mismatch must share an image and a 16x16-latent window
    # neighbourhood with a near-tie flip of an earlier slice
    other = ne & ~near_tie
    if other.any():
        ties = near_tie.nonzero()
        for b, c, y, x in other.nonzero().tolist():
            sl = c // (ref["symbols"].shape[1] // 4)
            ok = any(tb == b and tc // (ref["symbols"].shape[1] // 4) < sl and abs(ty - y) < 8 and abs(tx - x) < 8
                     for tb, tc, ty, tx in ties.tolist())
            assert ok, f"symbol mismatch at {(b, c, y, x)} is not a near-tie (|frac-0.5| = {dist[b, c, y, x]:.3e})"
    assert n / ne.numel() <= max_rate, f"{n} flipped symbols of {ne.numel()}"
    return n


def check_flip_sets_match(flipped_a: torch.Tensor, flipped_b: torch.Tensor, ref: dict, tie: float = 1e-6) -> int:
    """Two fp32-grade paths (e.g. exact-fp32 MFMA and fp32x6) flip the same symbols against the
    oracle, except (a) symbols whose oracle y - mu is within `tie` of the .5 boundary (a few fp32
    ulps: any two summation orders may round such a tie either way) and (b) their cascades -- a
    symbol of a later slice within the same 8-pixel latent neighbourhood of such a tie difference
    (a flipped y_hat of slice i moves mu of the later slices, net_ga.py:1021-1067).  Returns the
    size of the symmetric difference."""
    d = ref["z3"] - ref["means"]
    dist = ((d - torch.floor(d)) - 0.5).abs()
    diff = flipped_a ^ flipped_b
    ties = (diff & (dist < tie)).nonzero().tolist()
    per_slice = ref["symbols"].shape[1] // 4
    for b, c, y, x in (diff & (dist >= tie)).nonzero().tolist():
        ok = any(tb == b and tc // per_slice < c // per_slice and abs(ty - y) < 8 and abs(tx - x) < 8
                 for tb, tc, ty, tx in ties)
        assert ok, f"flip-set difference at {(b, c, y, x)} is neither an oracle tie nor its cascade " \
                   f"(|frac-0.5| = {dist[b, c, y, x]:.3e})"
    return int(diff.sum())


def _u8(x_rec):
    return torch.round(torch.clamp((x_rec.float().cpu() + 1) * 127.5, 0, 255)).to(torch.int32)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / b.abs().max()).item()


def check_decoder(last: dict, ref: dict, P: dict, flips: int, tol: float = 1e-4, M: int = 16):
    """Decoder side vs the oracle: the syntax vector before rounding, x_tilde = s_model(y_hat)
    and the uint8 reconstruction tanh(batch_conv(conv_weights_gen(round(syntax)), x_tilde)).
    With flipped near-tie symbols (check_symbols) y_hat differs locally, so the decoder is then
    pinned on the GPU's own y_hat / x_tilde through the oracle's s_model and recon head."""
    from oracle import ref_cpu as R
    assert _rel(last["syntax"], ref["syntax"]) < tol
    assert _u8(ref["x_rec"]).unique().numel() > 16            # the reconstruction is not degenerate
    if flips == 0:
        xt_ref, xr_ref = ref["x_tilde"], ref["x_rec"]
    else:
        xt_ref = R.synthesis_transform(last["y_hat"].float().cpu(), P)
        cw = R.conv_generator(torch.round(ref["syntax"]), P, "conv_weights_gen", M)
        xr_ref = torch.clamp(torch.tanh(R.batch_conv(cw, last["x_tilde"].float().cpu())), -1, 1)
    assert _rel(last["x_tilde"], xt_ref) < tol
    d8 = (_u8(last["x_rec"]) - _u8(xr_ref)).abs()
    assert int(d8.max()) <= 1 and (d8 > 0).float().mean().item() < 1e-4
