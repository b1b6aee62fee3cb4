"""The N>1 path on CPU: world_size-2 gloo process groups exercising the image
sharding, the MAX step-time reduction of bench.py and the single summary
all-reduce of eval_net.py (lic_amd.distributed)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from lic_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, _ = D.init("gloo")
    assert (r, w) == (rank, world)
    images = [f"img{i:02d}.png" for i in range(7)]
    mine = D.shard(images, r, w)
    # per-image statistics as eval_net.val accumulates them (time, bpp, psnr, mse, count)
    stats = [0.0, 0.0, 0.0, 0.0, 0.0]
    for name in mine:
        i = images.index(name)
        stats = [stats[0] + 0.01 * i, stats[1] + 0.5 + i, stats[2] + 30.0 + 0.25 * i, stats[3] + 2.0 * i, stats[4] + 1]
    total = D.sum_over_ranks(stats, w)
    D.barrier(w)
    tmax = D.max_over_ranks(1.5 + rank, w)
    q.put((rank, mine, total, tmax))
    D.finish(w)


def test_world2_shard_reduce_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    shards = [o[1] for o in out]
    images = [f"img{i:02d}.png" for i in range(7)]
    assert sorted(shards[0] + shards[1]) == images and not set(shards[0]) & set(shards[1])
    ref = [sum(0.01 * i for i in range(7)), sum(0.5 + i for i in range(7)), sum(30.0 + 0.25 * i for i in range(7)),
           sum(2.0 * i for i in range(7)), 7.0]
    for o in out:
        assert o[2] == pytest.approx(ref, rel=1e-12)
        assert o[3] == 2.5   # MAX over ranks of 1.5 + rank


def test_single_process_is_identity():
    assert D.shard([1, 2, 3], 0, 1) == [1, 2, 3]
    assert D.sum_over_ranks([1.0, 2.0], 1) == [1.0, 2.0]
    assert D.max_over_ranks(3.0, 1) == 3.0


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    D.init("gloo")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    unused = torch.nn.Linear(3, 3)                   # never receives a gradient
    params = list(model.parameters()) + list(unused.parameters())
    sync = D.GradAllReduce(params, world, bucket_mb=1e-4)   # tiny buckets: several in flight
    for step in range(2):
        for p in params:
            p.grad = None
        x = torch.randn(6, 8, generator=torch.Generator().manual_seed(100 * step + rank))
        model(x).pow(2).sum().backward()
        sync.finish()
    # numpy, not tensors: torch's fd-sharing pickler needs the child alive until the parent reads
    q.put((rank, [None if p.grad is None else p.grad.numpy().copy() for p in params]))
    D.finish(world)


def test_world2_grad_allreduce_gloo():
    """Bucketed gradient all-reduce of the training path: both ranks end with the mean of the
    per-rank gradients; parameters without a gradient stay None."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    grads = []
    for r in range(world):
        model.zero_grad()
        x = torch.randn(6, 8, generator=torch.Generator().manual_seed(100 + r))
        model(x).pow(2).sum().backward()
        grads.append([p.grad.clone() for p in model.parameters()])
    mean = [(a + b) / 2 for a, b in zip(*grads)]
    for r in range(world):
        got = out[r]
        for g_, m_ in zip(got[:4], mean):
            torch.testing.assert_close(torch.from_numpy(g_), m_, rtol=1e-5, atol=1e-6)
        assert got[4] is None and got[5] is None


def test_grad_allreduce_single_process_noop():
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    D.GradAllReduce([p], 1).finish()
    assert torch.equal(p.grad, torch.full((3,), 2.0))


def test_bench_launcher_two_ranks_dry_run():
    """`python bench.py --gpus 2` without torchrun starts its two ranks itself (gloo, --dry-run:
    no CUDA call), and rank 0's single JSON line reports n_gpus 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                         capture_output=True, text=True, timeout=180, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]   # (gloo logs its connections)
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["global_batch"] == 64 and rec["steps"] == 3 and rec["dry_run"]


def test_launch_workers_propagates_failure():
    """A failing rank stops the others and its exit status is returned."""
    import sys
    import time
    code = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['WORLD_SIZE'] == '3' and os.environ['LOCAL_RANK'] == str(r)\n"
            "assert os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
            "sys.exit(7) if r == 2 else time.sleep(60)\n")
    t0 = time.time()
    assert D.launch_workers([sys.executable, "-c", code], 3) == 7
    assert time.time() - t0 < 30
    ok = "import os; assert int(os.environ['WORLD_SIZE']) == 2"
    assert D.launch_workers([sys.executable, "-c", ok], 2) == 0


def test_bench_rejects_world_mismatch():
    """Under torchrun, --gpus must equal the launched world size."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode != 0 and "launcher started 1 ranks" in out.stderr
