"""Multi-GPU sharding: one process per GPU (torchrun), Monte-Carlo frames split by counter range,
ONE all-reduce of the int64 counters per sweep over RCCL (backend "nccl" on ROCm) or gloo (CPU
tests).  Counters are exact integers with per-frame quantised EVM, so the reduced result is
bit-identical for any world size."""
from __future__ import annotations

import os


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """[start, end) of the n units owned by `rank` (strong split; contiguous, balanced)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return n * rank // world, n * (rank + 1) // world


def weak_range(per_rank: int, rank: int) -> tuple[int, int]:
    """weak scaling: every rank owns per_rank units starting at rank * per_rank"""
    return rank * per_rank, (rank + 1) * per_rank


def env_rank_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def allreduce_counters(t):
    """Sum a counters tensor over all ranks in place (no-op when not distributed)."""
    import torch.distributed as dist  # noqa: PLC0415
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
