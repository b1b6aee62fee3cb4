"""The training gradient all-reduce (lic_amd/distributed.py GradAllReduce; replaces
the reference's nn.DataParallel gradient sum, train_net_unet.py:152) driven by the real liblic
autograd graph: two ranks on one GPU (gloo, CUDA tensors) train net_unet_ha_hs (bf16, as BASELINE
config 5) on different images; the post-accumulate-grad hooks must fire on the liblic model's
parameters, and after finish() both ranks hold bit-identical gradients equal to the mean of the
two ranks' local gradients of the same step (every liblic gradient reduction has a fixed order,
so each local gradient is reproducible)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from lic_amd import distributed as D
    from lic_amd.model import net_ga, net_unet_ha_hs
    D.init("gloo")
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    net = net_ga.synthetic_syntax_bias_(net_unet_ha_hs.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False,
                                                           precision="bf16")).to("cuda")
    params = net.base_params()
    x = (torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(50 + rank)) * 2 - 1).to("cuda")

    def step():
        for p in params:
            p.grad = None
        bpp, mse = net(x, "train", seed=7 + rank)
        (0.0025 * 255 ** 2 * mse + bpp).backward()

    step()                                              # local gradients of this rank
    local = [None if p.grad is None else p.grad.detach().float().cpu().numpy().copy() for p in params]
    sync = D.GradAllReduce(params, world, bucket_mb=4.0)
    fired = [0]
    for p in params:
        p.register_post_accumulate_grad_hook(lambda _p: fired.__setitem__(0, fired[0] + 1))
    step()                                              # same step, gradients all-reduced
    launched = sum(w is not None for w in sync._work)   # buckets launched from the hooks during backward
    sync.finish()
    synced = [None if p.grad is None else p.grad.detach().float().cpu().numpy().copy() for p in params]
    q.put((rank, local, synced, fired[0], launched, len(sync.buckets)))
    D.finish(world)


def test_grad_allreduce_on_liblic_model_two_ranks():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, local, synced, fired, launched, nb = q.get(timeout=240)
        out[r] = (local, synced, fired, launched, nb)
    for p in procs:
        p.join(timeout=60)
    (l0, s0, f0, la0, nb), (l1, s1, f1, la1, _) = out[0], out[1]
    import numpy as np
    n_grad = sum(g is not None for g in l0)
    print(f"\n[GradAllReduce, 2 ranks, net_unet_ha_hs bf16] {n_grad} gradients, {nb} buckets, hooks fired "
          f"{f0}/{f1}, buckets launched during backward {la0}/{la1}")
    assert n_grad > 300 and f0 >= n_grad and f1 >= n_grad
    assert la0 >= 1 and la1 >= 1                        # the all-reduce overlapped the backward
    for a, b, g0, g1 in zip(s0, s1, l0, l1):
        assert (a is None) == (g0 is None) == (b is None) == (g1 is None)
        if a is None:
            continue
        assert np.array_equal(a, b)                     # both ranks hold the same averaged gradient
        mean = (g0.astype(np.float32) + g1.astype(np.float32)) / np.float32(2)
        assert np.allclose(a, mean, rtol=0, atol=1e-6 * (np.abs(mean).max() + 1e-30))


def _graph_worker(port, q):
    """One rank with the RCCL ("nccl") backend: the training step with GradAllReduce's bucketed
    all-reduce (force=True runs the collective path at world 1) eager, and the same step captured
    in a hipGraph (train_net_unet.py --graph at world > 1) and replayed."""
    import copy
    import sys
    import torch.distributed as dist

    def say(msg):   # progress on stderr (a hang is located by the last line)
        print(f"[graph worker] {msg}", file=sys.stderr, flush=True)
    from lic_amd import distributed as D
    from lic_amd.model import net_ga, net_unet_ha_hs
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    say("process group up")
    torch.manual_seed(0)
    base = net_ga.synthetic_syntax_bias_(net_unet_ha_hs.Net((1, 256, 256, 3), (1, 256, 256, 3), False, False,
                                                            precision="bf16"))
    x = (torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(9)) * 2 - 1).to("cuda")
    steps = 3

    def make():
        net = copy.deepcopy(base).to("cuda")
        params = net.base_params()
        opt = torch.optim.Adam(params, lr=torch.tensor(1e-4, device="cuda"), capturable=True)
        sync = D.GradAllReduce(params, 1, bucket_mb=4.0, force=True)
        return net, params, opt, sync, torch.zeros((1,), dtype=torch.int64, device="cuda")

    def body(net, params, opt, sync, seed_t):
        bpp, mse = net(x, "train", seed_dev=seed_t)
        loss = 0.0025 * 255 ** 2 * mse + bpp
        loss.backward()
        sync.finish()
        torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], 1.0)
        opt.step()
        seed_t.add_(1)
        return loss.detach()

    net_a, pa, oa, sa_, ta = make()
    losses_a = []
    for _ in range(steps):
        oa.zero_grad(set_to_none=True)
        losses_a.append(body(net_a, pa, oa, sa_, ta).item())
        say(f"eager step {len(losses_a)}: loss {losses_a[-1]:.6f}")
    launched = len(sa_.buckets)
    net_b, pb, ob, sb_, tb = make()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ob.zero_grad(set_to_none=True)
        first = body(net_b, pb, ob, sb_, tb).item()
    torch.cuda.current_stream().wait_stream(side)
    say("warm-up step on the capture stream done")
    ob.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    sb_.defer = True   # collectives launched from finish() on this (capturing) thread
    g = torch.cuda.CUDAGraph()
    # as train_net_unet.py: thread_local capture (the process group's watchdog thread polls events)
    with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
        out = body(net_b, pb, ob, sb_, tb)
    say("captured")
    losses_b = [first]
    for _ in range(steps - 1):
        g.replay()
        losses_b.append(out.item())
        say(f"replay {len(losses_b) - 1}: loss {losses_b[-1]:.6f}")
    torch.cuda.synchronize()
    d = max(((p - q).norm() / (p.norm() + 1e-12)).item() for p, q in zip(net_a.parameters(), net_b.parameters()))
    q.put((losses_a, losses_b, d, launched))
    del g
    dist.destroy_process_group()


def test_graph_step_with_rccl_allreduce_matches_eager():
    """train_net_unet.py --graph at world > 1: the bucketed RCCL all-reduce is captured with the
    backward (a world-1 "nccl" group, collectives forced on); the replayed steps equal the eager
    steps bitwise (losses and every parameter)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_worker, args=(_free_port(), q))
    p.start()
    try:   # bounded: a hung collective fails the test instead of stalling the suite
        losses_a, losses_b, d, nb = q.get(timeout=150)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    print(f"\n[graph + RCCL all-reduce, {nb} buckets] eager losses {losses_a}, graph losses {losses_b}, "
          f"max relative parameter difference {d:.2e}")
    assert p.exitcode == 0
    assert losses_a == losses_b and d == 0
