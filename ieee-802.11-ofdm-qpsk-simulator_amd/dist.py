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


def allreduce_counters(t, word_stats: bool = False):
    """Sum a [n_snr][16] counters tensor over all ranks in place (no-op when not distributed).  With
    word_stats the OFDM_C_WL_* slots are extremes, not sums: MIN / MAX reduced, bits recomputed."""
    import torch.distributed as dist  # noqa: PLC0415
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return t
    if not word_stats:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t
    from . import abi  # noqa: PLC0415
    lo, hi = t[:, abi.C_WL_MIN_Q].clone(), t[:, abi.C_WL_MAX_Q].clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    t[:, abi.C_WL_MIN_Q], t[:, abi.C_WL_MAX_Q] = lo, hi
    t[:, abi.C_WL_BITS] = word_bits(lo, hi)
    return t


def word_bits(lo_q, hi_q):
    """integer bits of max(|min|, |max|) (OFDM.c:56-64) from the 2^-20 fixed-point extremes"""
    import torch  # noqa: PLC0415
    m = torch.maximum(lo_q.abs(), hi_q.abs()).double() / 2 ** 20
    b = torch.ceil(torch.log2(torch.clamp(m, min=1.0))).long() + 1
    return torch.where(m < 1.0, torch.ones_like(b), b)
