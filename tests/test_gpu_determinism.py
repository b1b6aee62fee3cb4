"""Bitwise determinism of the fp16 B=32 path the bench and the coder run (round-1 open
issue: 'decompress: corrupt bitstream' in ~1 of 4 coder_bench runs).

Root cause: the 8-wave window-attention kernel (attention_mfma.hip, used for fp16 maps with
>= 1024 windows, i.e. B >= 16 at 64x64) shared a token -> pixel table in LDS across its
waves; some launches read entries of that table that belonged to the previous workgroup
on the CU (a few windows of one image used a neighbouring window's pixels).  The table is
now computed per lane in registers and every LDS image of the kernel is wave-private.
These tests poison the caching allocator with fresh random values between calls (so the
memory layout and contents differ on every call) and require bit-identical results.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _poison():
    from determinism_probe import poison
    poison(1024, random=True)


def _net(B=32, precision="fp16"):
    from lic_amd.model import net_ga
    torch.manual_seed(0)
    return net_ga.Net((B, 256, 256, 3), (B, 256, 256, 3), False, False, precision=precision).to(DEV)


def _x(B=32, seed=1):
    return (torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(seed)) * 2 - 1).to(DEV)


def _bits(t):
    return t.view(torch.int16) if t.dtype == torch.float16 else (t.view(torch.int32) if t.dtype == torch.float32 else t)


def test_window_attention_8wave_chain_deterministic():
    """qkv GEMM -> 8-wave MFMA window attention -> proj on fresh buffers, 10 times."""
    from lic_amd.functional import Act
    net = _net()
    wba = net.a_model.transform[8].conv_b[0]
    x = Act((torch.randn(32, 64, 64, 192, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3)) * 0.5)
            .half())
    ref = wba.run(x).t.clone()
    for _ in range(10):
        _poison()
        assert torch.equal(_bits(wba.run(x).t), _bits(ref))


def test_forward_b32_fp16_bitwise_repeatable():
    net = _net()
    x = _x()
    net(x, "test", return_intermediates=True)
    ref = {k: v.clone() for k, v in net.last.items() if k in ("z3", "means", "scales", "symbols", "x_tilde")}
    for _ in range(3):
        _poison()
        net(x, "test", return_intermediates=True)
        for k, v in ref.items():
            assert torch.equal(_bits(net.last[k]), _bits(v)), k


def test_coder_b32_fp16_repeated_compress_then_decompress():
    """The failing sequence of tools/coder_bench.py: compress, several compress calls,
    then decompress the first bitstream twice; per-slice means / scales / y_hat of every
    decompress equal the first compress bit for bit."""
    net = _net()
    x = _x()
    net.update()
    enc = net.compress(x)
    c0 = {k: v.clone() for k, v in net.last_coder.items()}
    for _ in range(4):
        _poison()
        e2 = net.compress(x)
        assert e2["strings"] == enc["strings"]
    for _ in range(2):
        _poison()
        d = net.decompress(enc["strings"], enc["shape"], enc["syntax"])
        assert torch.equal(d["symbols"], enc["symbols"])
        for k in ("means", "scales", "y_hat", "z_hat"):
            assert torch.equal(_bits(net.last_coder[k]), _bits(c0[k])), k
