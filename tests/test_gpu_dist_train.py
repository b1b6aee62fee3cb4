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
