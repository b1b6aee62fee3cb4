"""hipGraph capture of the one-level stream forks the forward uses (net_ga.py's hyper / slice /
syntax side streams: main -> side, joined back), with liblic convolutions on both streams: the
replay must equal the eager run bit for bit.  The nested fork (a side stream forked from a side
stream) segfaults in capture_end even with plain torch kernels (tools/capture_fork_probe.py), so the
model keeps its forks one level deep."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("pattern", ["flat", "sibling"])
@pytest.mark.parametrize("use_lic", [False, True])
def test_capture_one_level_forks(pattern, use_lic):
    import capture_fork_probe as P
    assert P.run(pattern, use_lic, "global")


@pytest.mark.parametrize("precision", ["fp32x6", "fp16"])
def test_conv_a_fork_bitwise(precision, monkeypatch):
    """The model's conv_a forks (Win_noShift_Attention at the 16x16 latents of the a_model / s_model, the
    slice loop's mean SWAtten: a side stream forked from the capture stream, a sibling of the slice loop's
    scale-branch stream -- never nested) change nothing: eager with and without the forks and the hipGraph
    replay with them give the same bits."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    B, S = 4, 256
    net = bench.build_net("net_ga", precision, S, B, "cpu").cuda()
    x = bench.bench_input(B, S, 0).cuda()
    outs = {}
    for fork in ("0", "1"):
        monkeypatch.setenv("LIC_FORK_CONV_A", fork)
        for _ in range(2):
            r = net(x, "test", return_intermediates=True)
        torch.cuda.synchronize()
        outs[fork] = ([t.clone() for t in r], net.last["symbols"].clone(), net.last["x_tilde"].clone(),
                      net.last["means"].clone())
    a, b = outs["0"], outs["1"]
    assert all(torch.equal(u, v) for u, v in zip(a[0], b[0]))
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
    # captured with the forks, replayed
    g, out = bench.capture(lambda: net(x, "test"))
    g.replay()
    torch.cuda.synchronize()
    assert all(torch.equal(u, v) for u, v in zip(out, b[0]))


@pytest.mark.parametrize("precision", ["fp32x6", "fp16"])
def test_analysis_chains_match(precision, monkeypatch):
    """LIC_CHAINS=2 (opt-in: two half-batches of the analysis transform on two streams, forked from the
    current stream and joined back) computes the same latents as the single chain: images are independent,
    only the launch split differs (a launch on a half-batch may pick another tiling, so equality is to
    accumulation-order tolerance, not bitwise), and it captures into a hipGraph."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from lic_amd.functional import Act, split_f32
    B, S = 8, 256
    dt = torch.float16 if precision == "fp16" else torch.float32
    net = bench.build_net("net_ga", precision, S, B, "cpu").cuda()
    x = bench.bench_input(B, S, 0).cuda()
    xin = Act(x.to(dt).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1))
    ys = {}
    with torch.no_grad(), split_f32(bench.SPLIT_MODES.get(precision, 0)):
        for n in ("1", "2"):
            monkeypatch.setenv("LIC_CHAINS", n)
            ys[n] = net.a_model.run(xin).t.float().clone()
        g, out = bench.capture(lambda: net.a_model.run(xin))
        g.replay()
    torch.cuda.synchronize()
    ref = ys["1"]
    tol = (2e-2 if precision == "fp16" else 1e-4) * ref.abs().max().item()
    assert (ys["2"] - ref).abs().max().item() <= tol
    assert torch.equal(out.t.float(), ys["2"])
