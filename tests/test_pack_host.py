"""CPU: the strided-view weight packs (one casting copy per phase) hold exactly the bytes, taps
and offsets of the per-tap gather they replaced -- the stride-s dgrad packs
(lic_amd.autograd.dgrad_packs) and the transposed-conv phase packs (functional.pack_conv_transpose2d)."""
import pytest
import torch

import lic_amd.autograd as AG
import lic_amd.functional as Fn


def _dgrad_per_tap(weight, s, pad, dtype, co_pad):
    co, ci, kh, kw = weight.shape
    pt, pl = pad[0], pad[1]
    out = []
    for ry in range(s):
        for rx in range(s):
            taps = [(ky, kx) for ky in range(kh) for kx in range(kw)
                    if (ry - (ky - pt)) % s == 0 and (rx - (kx - pl)) % s == 0]
            if not taps:
                continue
            w = torch.zeros((Fn._choose_copad(ci), len(taps), Fn._cpad_for(co_pad, dtype)), dtype=dtype)
            for t, (ky, kx) in enumerate(taps):
                w[:ci, t, :co] = weight[:, :, ky, kx].t().to(dtype)
            out.append((w, [(ry - (ky - pt)) // s for ky, kx in taps], [(rx - (kx - pl)) // s for ky, kx in taps]))
    return out


def _convt_per_tap(weight, s, p, dtype, prepad):
    ci, co, kh, kw = weight.shape
    out = []
    for ry in range(s):
        for rx in range(s):
            kys = [ky for ky in range(kh) if (ry + p - ky) % s == 0]
            kxs = [kx for kx in range(kw) if (rx + p - kx) % s == 0]
            taps = [(ky, kx) for ky in sorted(kys, reverse=True) for kx in sorted(kxs, reverse=True)]
            if not taps:
                continue
            w = torch.zeros((Fn._choose_copad(co), len(taps), Fn._cpad_for(ci, dtype)), dtype=dtype)
            for t, (ky, kx) in enumerate(taps):
                w[:co, t, :ci] = weight[:, :, ky, kx].t().to(dtype)
            out.append((w, [(ry + p - ky) // s - prepad[0] for ky, kx in taps],
                        [(rx + p - kx) // s - prepad[1] for ky, kx in taps]))
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("co,ci,k,s,pad", [
    (16, 8, 3, 2, (1, 1, 1, 1)), (40, 24, 5, 2, (1, 1, 2, 2)), (24, 40, 5, 2, (2, 2, 2, 2)),
    (192, 3, 3, 2, (0, 0, 1, 1)), (8, 8, 7, 3, (3, 2, 3, 3)), (8, 16, 4, 2, (1, 1, 2, 2)),
])
def test_dgrad_packs_match_per_tap(dtype, co, ci, k, s, pad):
    g = torch.Generator().manual_seed(co * 7 + ci + k)
    w = torch.randn(co, ci, k, k, generator=g)
    co_pad = Fn._cpad_for(co, dtype)
    ref = _dgrad_per_tap(w, s, pad, dtype, co_pad)
    got = AG.dgrad_packs(w, s, pad, dtype, co_pad)
    assert len(got) == len(ref)
    for pk, (rw, rdy, rdx) in zip(got, ref):
        assert pk.w.dtype == dtype and pk.w.shape == rw.shape
        assert torch.equal(pk.w, rw)
        assert list(pk.dy) == rdy and list(pk.dx) == rdx


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("ci,co,k,s,p,prepad", [
    (192, 192, 5, 2, 3, (1, 1)), (24, 40, 5, 2, 2, (0, 0)), (16, 3, 5, 2, 2, (1, 1)),
    (8, 16, 3, 2, 1, (0, 0)), (8, 8, 4, 2, 1, (1, 0)), (16, 8, 7, 3, 2, (0, 0)),
])
def test_convt_packs_match_per_tap(dtype, ci, co, k, s, p, prepad):
    g = torch.Generator().manual_seed(ci * 5 + co + k)
    w = torch.randn(ci, co, k, k, generator=g)
    ref = _convt_per_tap(w, s, p, dtype, prepad)
    got = Fn.pack_conv_transpose2d(w, None, s, p, 1 if s == 2 else 0, dtype, prepad)
    assert len(got) == len(ref)
    for pk, (rw, rdy, rdx) in zip(got, ref):
        assert pk.w.dtype == dtype and pk.w.shape == rw.shape
        assert torch.equal(pk.w, rw)
        assert list(pk.dy) == rdy and list(pk.dx) == rdx
