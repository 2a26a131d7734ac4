"""Multi-process path on CPU (gloo, world_size 2 and 4): counter-range sharding + ONE all-reduce of the
int64 counters gives exactly the single-process result.  Per-rank counters come from
the oracle (test data source); the GPU ranks use the same dist helpers over RCCL."""
import json
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, n, snrs, out_path):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ofdm_pkg
    ofdm_pkg.load()
    from ofdm_amd import dist as odist
    from oracle import Oracle
    O = Oracle()
    r, w, _ = odist.env_rank_world()
    assert (r, w) == (rank, world)
    if mode == "strong":
        a, b = odist.shard_range(n, rank, world)
    else:
        a, b = odist.weak_range(n // world, rank)
    c = O.symbol_sweep(O.cfg(), snrs, a, b - a)
    t = torch.from_numpy(c)
    odist.allreduce_counters(t)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world,n", [("strong", 2, 96), ("weak", 2, 96), ("strong", 4, 101), ("weak", 4, 100)])
def test_ranks_allreduce_equals_single(tmp_path, oracle, mode, world, n):
    """world 2, and world 4 (a rehearsal of more ranks than the one-GPU box can run over RCCL) with a frame count
    the strong split cannot divide evenly: the summed shards equal one process's sweep bit for bit"""
    snrs = [0.0, 4.0, 8.0]
    out = tmp_path / "c.npy"
    mp.spawn(_worker, args=(world, _free_port(), mode, n, snrs, str(out)), nprocs=world, join=True)
    got = np.load(out)
    ref = oracle.symbol_sweep(oracle.cfg(), snrs, 0, n if mode == "strong" else (n // world) * world)
    assert np.array_equal(got, ref)


def _wl_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ofdm_pkg
    ofdm_pkg.load()
    from ofdm_amd import abi, dist as odist
    t = torch.zeros((2, 16), dtype=torch.int64)
    t[:, abi.C_BITS] = 100 * (rank + 1)
    t[:, abi.C_WL_MIN_Q] = torch.tensor([-3 << 20, -1 << 19]) * (rank + 1)      # rank 1 holds the minimum
    t[:, abi.C_WL_MAX_Q] = torch.tensor([5 << 20, 1 << 18]) * (2 - rank)        # rank 0 holds the maximum
    odist.allreduce_counters(t, word_stats=True)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_word_stats_reduce_min_max(tmp_path):
    """OFDM_C_WL_* slots are extremes: MIN / MAX over ranks, bits recomputed; everything else sums."""
    out = tmp_path / "w.npy"
    mp.spawn(_wl_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    t = np.load(out)
    assert list(t[:, 2]) == [300, 300]
    assert list(t[:, 13]) == [-6 << 20, -1 << 20] and list(t[:, 14]) == [10 << 20, 1 << 19]
    assert list(t[:, 15]) == [5, 1]           # max|.| 10 -> ceil(log2 10) + 1 = 5; 1.0 -> ceil(0) + 1 = 1


def _late_rank0_worker(rank, world, port, out_path):
    """bench.py's order under torchrun: rank 0 times the reference BEFORE it forms the process group (here a
    real, short cpu_baseline on 2 host processes), the other rank goes straight to init_process_group and
    waits at the rendezvous; then the counters' all-reduce runs as usual."""
    import sys
    import time
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import argparse
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    sys.modules["bench"] = bench
    spec.loader.exec_module(bench)
    cpu = None
    t0 = time.perf_counter()
    if bench.wants_cpu_baseline(argparse.Namespace(no_cpu_baseline=False)):
        share = {"cores": 2, "affinity": 2, "quota": None, "source": "test", "visible": 2}
        cpu = bench.cpu_baseline("c3", seconds=0.5, share=share)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    waited = time.perf_counter() - t0
    t = torch.full((2, 16), rank + 1, dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        np.save(out_path, t.numpy())
        Path(out_path).with_suffix(".json").write_text(json.dumps({"cpu": cpu}))
    else:
        np.save(str(out_path) + f".{rank}.npy", np.array([waited]))
    dist.barrier()
    dist.destroy_process_group()


def test_rank0_times_the_reference_before_the_rendezvous(tmp_path, reflib):
    out = tmp_path / "late.npy"
    mp.spawn(_late_rank0_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert np.array_equal(np.load(out), np.full((2, 16), 3))
    cpu = json.loads(out.with_suffix(".json").read_text())["cpu"]
    assert cpu["kind"] == "reference" and cpu["cores"] == 2 and cpu["value"] > 0
    assert np.load(str(out) + ".1.npy")[0] > 0.3          # rank 1 waited at the rendezvous for rank 0
