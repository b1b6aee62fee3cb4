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
