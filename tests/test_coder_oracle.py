"""CPU: the entropy-coder oracle (oracle/rans_ref.c + oracle/ref_coder.py, a restatement
of compressai 1.2.x's pmf_to_quantized_cdf and Rans64 encode/decode_with_indexes).

compressai is not importable here and ships no fixtures, so parity with compressai is
UNPINNED; the oracle is pinned by hand-derived known answers and round trips."""
import numpy as np
import pytest
import torch

from oracle import ref_coder as C


def test_pmf_to_cdf_known_answers():
    assert C.pmf_to_quantized_cdf([0.25, 0.25, 0.5]).tolist() == [0, 16384, 32768, 65536]
    # a zero-probability symbol steals one count from the only frequency > 1
    assert C.pmf_to_quantized_cdf([1.0, 0.0]).tolist() == [0, 65535, 65536]
    # rounding then renormalisation: round(p * 2^16) / total
    assert C.pmf_to_quantized_cdf([0.5, 0.5, 0.5, 0.5]).tolist() == [0, 16384, 32768, 49152, 65536]


def test_rans_encode_known_answer():
    # one table {symbol 0: freq 32768, tail: 32768}; x = 2^31 -> (2^31 / 2^15) << 16 = 2^32
    cdf = np.array([[0, 32768, 65536]], dtype=np.int32)
    w = C.encode(np.array([0]), np.array([0]), cdf, np.array([3], np.int32), np.array([0], np.int32))
    assert w.tolist() == [0, 1]
    # an empty symbol list is just the flushed initial state
    w0 = C.encode(np.zeros(0, np.int32), np.zeros(0, np.int32), cdf, np.array([3], np.int32),
                  np.array([0], np.int32))
    assert w0.tolist() == [1 << 31, 0]


def test_gauss_tables_are_valid_cdfs():
    cdf, sizes, offsets = C.gauss_tables()
    st = C.get_scale_table()
    assert cdf.shape[0] == 64 and len(sizes) == 64
    assert sizes[0] == 5 and offsets[0] == -1          # s = 0.11: ceil(0.11 * 6.109) = 1
    assert sizes[-1] == 2 * int(np.ceil(256 * 6.1094102048693975)) + 3
    for t in range(64):
        row = cdf[t, :sizes[t]]
        assert row[0] == 0 and row[-1] == 65536
        assert (np.diff(row) > 0).all()                 # every symbol (and the tail) codable
    # wider scales spread mass: the centre frequency decreases with the scale
    centre = [int(cdf[t, -offsets[t] + 1] - cdf[t, -offsets[t]]) for t in range(64)]
    assert all(a >= b for a, b in zip(centre, centre[1:]))
    assert float(st[0]) == pytest.approx(0.11) and float(st[-1]) == pytest.approx(256, rel=1e-6)


def test_build_indexes_matches_definition():
    st = C.get_scale_table()
    s = torch.tensor([0.0, 0.11, 0.1100001, 1.0, 255.9, 256.0, 300.0])
    idx = C.build_indexes(s, st)
    s32 = np.maximum(s.numpy(), np.float32(0.11))
    ref = [int(np.searchsorted(st.numpy()[:-1], v, side="left")) for v in s32]
    assert idx.tolist() == ref


@pytest.mark.parametrize("seed", [0, 1])
def test_rans_round_trip_with_bypass(seed):
    cdf, sizes, offsets = C.gauss_tables()
    rng = np.random.default_rng(seed)
    n = 1000
    idx = rng.integers(0, 64, n).astype(np.int32)
    sym = np.round(rng.normal(0, 1, n) * np.exp(idx / 12.0)).astype(np.int32)
    sym[::97] = rng.integers(-(1 << 24), 1 << 24, len(sym[::97]))   # far outside every table: bypass
    sym[5], sym[6] = np.int32(2 ** 30), np.int32(-2 ** 30)
    w = C.encode(sym, idx, cdf, sizes, offsets)
    assert (C.decode(w, idx, cdf, sizes, offsets) == sym).all()


def test_eb_tables_default_init():
    from lic_amd.layers.compressai import EntropyBottleneck
    torch.manual_seed(0)
    eb = EntropyBottleneck(8)
    P = {"entropy_bottleneck." + k: v.detach() for k, v in eb.state_dict().items()}
    P.update({"entropy_bottleneck." + k: v.detach() for k, v in eb.named_parameters()})
    cdf, sizes, offsets, medians = C.eb_tables(P)
    assert (sizes == 23).all() and (offsets == -10).all()          # quantiles [-10, 0, 10]
    for t in range(8):
        row = cdf[t, :sizes[t]]
        assert row[0] == 0 and row[-1] == 65536 and (np.diff(row) > 0).all()
    sym = np.random.default_rng(3).integers(-30, 30, (2, 4, 4, 8)).astype(np.int32)
    words, offs = C.encode_latent(sym, None, cdf, sizes, offsets)
    for b in range(2):
        for c in range(8):
            s = b * 8 + c
            got = C.decode(words[offs[s]:offs[s + 1]], np.full(16, c, np.int32), cdf, sizes, offsets)
            assert (got == sym[b, :, :, c].ravel()).all()
