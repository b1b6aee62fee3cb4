"""Multi-GPU plumbing for the encode -> quantize -> decode path.

Images are independent units: one process per GPU (``torch.distributed.run``),
images sharded round-robin over ranks, no exchange on the data path.  The only
collectives are a barrier around timed regions, a MAX of the elapsed time
(bench.py) and ONE all-reduce of a small fp64 statistics vector per evaluation
(eval_net.py: sum of bpp, PSNR, MSE, time and the image count) so that rank 0
prints exactly the single-process summary.  Backend "nccl" (RCCL over xGMI) on
the GPU box, "gloo" for the CPU tests.  ``bench.py --gpus N`` / ``eval_net.py --gpus N``
started without torchrun spawn their N ranks themselves (``launch_workers``).
"""
from __future__ import annotations

import os
import signal
import threading
import socket
import subprocess
import sys
import time
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def launched() -> bool:
    """True inside a worker of torchrun or of ``launch_workers`` (WORLD_SIZE is set)."""
    return "WORLD_SIZE" in os.environ


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(cmd: Sequence[str], n: int, poll_s: float = 0.2) -> int:
    """Run ``cmd`` as ``n`` worker processes, one per GPU, the way ``torch.distributed.run
    --nnodes 1 --nproc-per-node n`` would: each child gets RANK = LOCAL_RANK = i, WORLD_SIZE =
    LOCAL_WORLD_SIZE = n and MASTER_ADDR / MASTER_PORT of a local rendezvous; the child selects
    its device from LOCAL_RANK.  The caller must not have touched the GPU (the children are new
    programs started with fork + exec of a fresh interpreter; nothing GPU-initialised is ever
    replaced).  Rank 0's stdout is this process's stdout (the single JSON line of bench.py /
    eval_net.py); the other ranks' stdout goes to stderr.  When any child fails the others are
    terminated; returns the first non-zero exit status (0 when every rank succeeded)."""
    if n < 1:
        raise ValueError(f"need at least one worker, got {n}")
    # the launcher hosts the rendezvous store itself, the way torchrun's agent does: it binds an
    # ephemeral port and keeps it for the children's lifetime (no probe-then-release race), and the
    # ranks' env:// rendezvous connects to it as clients (TORCHELASTIC_USE_AGENT_STORE)
    store = dist.TCPStore("127.0.0.1", 0, n, True, wait_for_workers=False)
    port = store.port
    procs = []

    def _stop(signum, frame):   # SIGTERM / SIGINT to the launcher: take the ranks down with it
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise SystemExit(128 + signum)

    # signal.signal works in the main thread only; from a worker thread the finally block's kill is the
    # only clean-up
    old = ({sig: signal.signal(sig, _stop) for sig in (signal.SIGTERM, signal.SIGINT)}
           if threading.current_thread() is threading.main_thread() else {})
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       TORCHELASTIC_USE_AGENT_STORE="True")
            # ranks > 0 write their stdout to the launcher's stderr descriptor (fd 2 works whatever
            # object sys.stderr is, e.g. under pytest capture)
            procs.append(subprocess.Popen(list(cmd), env=env, stdout=None if r == 0 else 2))
        status = 0
        live = set(range(n))
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = rc
                    print(f"launch_workers: rank {r} exited with status {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        procs[q].terminate()
            if live:
                time.sleep(poll_s)
        return status
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1-process defaults)."""
    def _i(k, d):
        try:
            return int(os.environ.get(k, d))
        except ValueError:
            return d
    return _i("RANK", 0), _i("WORLD_SIZE", 1), _i("LOCAL_RANK", 0)


def init(backend: str = "nccl") -> Tuple[int, int, int]:
    """Join the process group when launched with WORLD_SIZE > 1; returns (rank, world, local)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, init_method="env://")
    return rank, world, local


def shard(items: Sequence, rank: int, world: int) -> List:
    """Round-robin share of `items` for `rank` (item i -> rank i % world)."""
    return [it for i, it in enumerate(items) if i % world == rank]


def barrier(world: int) -> None:
    if world > 1:
        dist.barrier()


def max_over_ranks(value: float, world: int, device=None) -> float:
    """MAX of a per-rank scalar (the step-time reduction of bench.py)."""
    if world <= 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(stats: Sequence[float], world: int, device=None) -> List[float]:
    """Element-wise SUM of a small per-rank statistics vector (one all-reduce)."""
    if world <= 1:
        return [float(v) for v in stats]
    t = torch.tensor(list(stats), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def finish(world: int) -> None:
    if world > 1 and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


class GradAllReduce:
    """Data-parallel gradient averaging for the training path (replaces the
    reference's single-process ``nn.DataParallel`` gradient sum, train_net_unet.py:152).

    One process per GPU; parameters are grouped into ~``bucket_mb`` buckets in reverse
    registration order (roughly the order backward produces their gradients).  A
    post-accumulate-grad hook counts each bucket down; when its last gradient lands the
    bucket is flattened and an async all-reduce (SUM) is launched on it (RCCL over xGMI),
    overlapping the rest of the backward.  ``finish()`` launches what is left (buckets
    holding parameters that got no gradient this step: only the ones that did are reduced,
    the same set on every rank because every rank runs the same graph), waits, divides by
    the world size and scatters back into ``.grad``.

    Every step of it is stream-ordered (flatten, RCCL all-reduce on the communicator's stream
    joined through events, wait, scale, scatter), so a training step that calls ``finish()``
    inside ``torch.cuda.graph`` captures the collectives too: replays run the bucketed all-reduce
    with no host work (train_net_unet.py --graph at world > 1).  ``force`` runs the collective
    path at world 1 as well (a one-rank all-reduce: the graph-capture test of the path).

    ``defer = True`` (set around a hipGraph capture) launches every bucket from ``finish()`` on the
    capturing thread instead of from the backward's hooks: a collective issued from the autograd
    thread is queued to the process group's watchdog, whose event queries then fail on events
    recorded in a capturing stream (hipErrorCapturedEvent, seen on MI355X).  The replays run the
    same collectives with no host work either way."""

    def __init__(self, params, world: int, bucket_mb: float = 32.0, force: bool = False):
        self.world = world
        self.active = world > 1 or force
        self.params = [p for p in params if p.requires_grad]
        buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_mb * 2 ** 20:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        self.buckets = buckets
        self._where = {id(p): i for i, b in enumerate(buckets) for p in b}
        self._pending = [len(b) for b in buckets]
        self._work = [None] * len(buckets)
        self._flat = [None] * len(buckets)
        self._members = [None] * len(buckets)
        self._hooks = []
        self.defer = False
        if self.active:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _on_grad(self, p):
        i = self._where[id(p)]
        self._pending[i] -= 1
        if self._pending[i] == 0 and not self.defer:
            self._launch(i)

    def _launch(self, i):
        members = [p for p in self.buckets[i] if p.grad is not None]
        self._members[i] = members
        if not members:
            return
        flat = torch.cat([p.grad.reshape(-1).float() for p in members])
        self._flat[i] = flat
        self._work[i] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)

    def finish(self) -> None:
        """Complete every bucket's all-reduce and write the averaged gradients back."""
        if not self.active:
            return
        for i in range(len(self.buckets)):
            if self._members[i] is None:
                self._launch(i)
            if self._work[i] is not None:
                self._work[i].wait()
                flat = self._flat[i].div_(self.world)
                off = 0
                for p in self._members[i]:
                    n = p.numel()
                    p.grad.copy_(flat[off:off + n].view_as(p.grad))
                    off += n
            self._pending[i] = len(self.buckets[i])
            self._work[i] = self._flat[i] = self._members[i] = None
