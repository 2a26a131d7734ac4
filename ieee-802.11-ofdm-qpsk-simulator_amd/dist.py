"""Multi-GPU sharding: one process per GPU (torchrun), Monte-Carlo frames split by counter range,
ONE all-reduce of the int64 counters per sweep over RCCL (backend "nccl" on ROCm) or gloo (CPU
tests, or several ranks sharing one GPU).  Counters are exact integers with per-frame quantised
EVM, so the reduced result is bit-identical for any world size.

The reference has no parallelism at all (src/OFDM.c:1187-1222 is one single-threaded loop): the
trial loop it runs per SNR point is what gets sharded here."""
from __future__ import annotations

import os


class DistError(RuntimeError):
    pass


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


def init_from_env(backend: str | None = None, device: int | None = None) -> bool:
    """Form the process group of a torchrun launch (RANK / WORLD_SIZE / MASTER_* in the
    environment).  backend None: $OFDM_DIST_BACKEND, else "nccl" (RCCL over xGMI, one rank per GPU).
    "gloo" keeps the counters on the host (CPU tests, several ranks on one GPU).  Returns True when
    a group of more than one rank exists afterwards; a no-op outside torchrun."""
    import torch.distributed as dist  # noqa: PLC0415
    rank, world, local = env_rank_world()
    if "RANK" not in os.environ or not dist.is_available():
        return False
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or os.environ.get("OFDM_DIST_BACKEND", "nccl")
        if backend == "nccl":
            import torch  # noqa: PLC0415
            dev = local if device is None else device
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return dist.get_world_size() > 1


def _require_group(world_env: int):
    import torch.distributed as dist  # noqa: PLC0415
    ok = dist.is_available() and dist.is_initialized()
    if world_env > 1 and not ok:
        # a sharded sweep reduced on one rank only would write that rank's share as the result
        raise DistError(f"WORLD_SIZE={world_env} but no process group: call dist.init_from_env() first")
    return ok and dist.get_world_size() > 1


def allreduce_counters(t, word_stats: bool = False):
    """Sum a [n_snr][16] counters tensor over all ranks in place.  A no-op for one process; raises
    when WORLD_SIZE > 1 and no process group was formed.  With word_stats the OFDM_C_WL_* slots are
    extremes, not sums: MIN / MAX reduced, bits recomputed."""
    import torch.distributed as dist  # noqa: PLC0415
    if not _require_group(int(os.environ.get("WORLD_SIZE", 1))):
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


def allreduce_counters_np(c, device: int = 0, word_stats: bool = False):
    """allreduce_counters for a host int64 array: through HBM on the nccl backend, in host memory on
    gloo.  Returns the reduced array (a new one when a reduction ran)."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415
    if not _require_group(int(os.environ.get("WORLD_SIZE", 1))):
        return c
    t = torch.from_numpy(c.copy())
    if dist.get_backend() == "nccl":
        t = t.to(f"cuda:{device}")
    allreduce_counters(t, word_stats=word_stats)
    return t.cpu().numpy()


def word_bits(lo_q, hi_q):
    """integer bits of max(|min|, |max|) (OFDM.c:56-64) from the 2^-20 fixed-point extremes"""
    import torch  # noqa: PLC0415
    m = torch.maximum(lo_q.abs(), hi_q.abs()).double() / 2 ** 20
    b = torch.ceil(torch.log2(torch.clamp(m, min=1.0))).long() + 1
    return torch.where(m < 1.0, torch.ones_like(b), b)
