"""Host-side layout of the packed split weights (csrc/conv_split.h): MFMA-fragment order
[copad/32][cpad/16][ntaps][part][64 lanes][8], lane = 32 * (channel half) + (co % 32), and the
exact three-part bf16 / two-part fp16 splits (no GPU needed)."""
import torch

import lic_amd.functional as Fn


def test_frag_order_element_mapping_and_inverse():
    g = torch.Generator().manual_seed(5)
    parts = [torch.randn(64, 9, 32, generator=g).to(torch.bfloat16) for _ in range(3)]
    P = Fn._frag_order(parts)
    assert P.shape == (2, 2, 9, 3, 64, 8)
    for (j, k, t, p, lane, e) in [(0, 0, 0, 0, 0, 0), (1, 1, 8, 2, 63, 7), (0, 1, 4, 1, 37, 3), (1, 0, 2, 0, 31, 5)]:
        co, ci = 32 * j + lane % 32, 16 * k + 8 * (lane // 32) + e
        assert P[j, k, t, p, lane, e] == parts[p][co, t, ci]
    back = Fn.split_weights_parts(P)
    for p in range(3):
        assert torch.equal(back[p], parts[p])


def test_split_weights_exact_parts():
    g = torch.Generator().manual_seed(6)
    w = torch.randn(64, 9, 48, generator=g) * torch.logspace(-6, 0.5, 48)
    pk = Fn.ConvPack.__new__(Fn.ConvPack)
    pk.__dict__["w"] = w
    ws = Fn.split_weights(pk, 2)
    parts = Fn.split_weights_parts(ws).float()
    assert torch.equal(parts.sum(0), w)             # three bf16 parts carry all 24 bits
    assert ws.dtype == torch.bfloat16
    w1 = Fn.split_weights(pk, 1)                    # fp16 W1 + W2 = 2^11 w to ~2^-22
    p1 = Fn.split_weights_parts(w1).float()
    err = ((p1.sum(0) / 2048.0 - w).abs() / w.abs().clamp_min(1e-3)).max().item()
    assert err < 1e-6
    assert Fn.split_weights(pk, 2) is ws            # cached on the pack


def test_stride2_phase_packs_partition_taps():
    """ZeroPad2d((1,2,1,2)) + conv5x5 s2 (net_ga.py:277-282): the four parity phases hold 9, 6, 6, 4
    taps, every tap exactly once, each phase's offsets share one row and one column parity, the
    bias only in the first; phases are not split again."""
    pk = Fn.ConvPack.__new__(Fn.ConvPack)
    dy = [y for y in range(-1, 4) for x in range(-1, 4)]
    dx = [x for y in range(-1, 4) for x in range(-1, 4)]
    pk.__dict__.update(w=torch.randn(64, 25, 32), bias=torch.randn(64), ci=32, co=64, dy=dy, dx=dx, groups=1,
                       stride=2, pad=(1, 1, 2, 2), kh=5, kw=5, phase=None)
    ph = Fn.stride2_phase_packs(pk)
    assert [len(p.dy) for p in ph] == [9, 6, 6, 4]
    seen = sorted((y, x) for p in ph for y, x in zip(p.dy, p.dx))
    assert seen == sorted(zip(dy, dx))
    for p in ph:
        assert len({(y + 1) % 2 for y in p.dy}) == 1 and len({(x + 1) % 2 for x in p.dx}) == 1
        for t, (y, x) in enumerate(zip(p.dy, p.dx)):
            assert torch.equal(p.w[:, t], pk.w[:, dy.index(y) * 0 + [i for i in range(25) if dy[i] == y and dx[i] == x][0]])
    assert ph[0].bias is pk.bias and all(p.bias is None for p in ph[1:])
    assert Fn.stride2_phase_packs(ph[0]) is None
    assert Fn.stride2_phase_packs(pk) is ph      # cached
