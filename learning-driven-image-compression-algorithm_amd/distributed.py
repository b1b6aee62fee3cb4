"""Multi-GPU plumbing for the encode -> quantize -> decode path.

Images are independent units: one process per GPU (``torch.distributed.run``),
images sharded round-robin over ranks, no exchange on the data path.  The only
collectives are a barrier around timed regions, a MAX of the elapsed time
(bench.py) and ONE all-reduce of a small fp64 statistics vector per evaluation
(eval_net.py: sum of bpp, PSNR, MSE, time and the image count) so that rank 0
prints exactly the single-process summary.  Backend "nccl" (RCCL over xGMI) on
the GPU box, "gloo" for the CPU tests.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


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
