"""Multi-process path on CPU (gloo, world_size 2): counter-range sharding + ONE all-reduce of the
int64 counters gives exactly the single-process result.  Per-rank counters come from
the oracle (test data source); the GPU ranks use the same dist helpers over RCCL."""
import os
import socket

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


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_two_rank_allreduce_equals_single(tmp_path, oracle, mode):
    snrs = [0.0, 4.0, 8.0]
    n = 96
    out = tmp_path / "c.npy"
    mp.spawn(_worker, args=(2, _free_port(), mode, n, snrs, str(out)), nprocs=2, join=True)
    got = np.load(out)
    ref = oracle.symbol_sweep(oracle.cfg(), snrs, 0, n)
    assert np.array_equal(got, ref)
