"""Multi-rank paths through the HIP library (BASELINE configs[3] C4 / configs[4] C5).

* C4's per-rank shard at its stated size (1e8 symbols/point over 8 ranks = 1.25e7 per rank) equals
  the sum of its two halves bit for bit (counter-range sharding of OFDM.c's trial loop :1195-1222).
* C4's and C5's whole jobs, split 8 / 4 / 2 ways by shard_range and run rank after rank on this
  device ("fake ranks"), sum to the single-range sweep bit for bit.
* Two spawned processes on cuda:0 run Engine.symbol_sweep / sweep.reference_main on their shard
  and reduce through dist.allreduce_counters over gloo: bit-identical to one process.
* torchrun launches bench.py as a fresh child, so init_process_group("nccl") and the RCCL
  all-reduce of the counters run on the MI355X.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

SNR = np.arange(0.0, 31.0, 2.0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c4_rank_shard_equals_halves(engine, pkg):
    """C4: 1e8 symbols/point on 8 GPUs -> one rank's 1.25e7 symbols/point (6.25e6 frames), here rank 3."""
    from ofdm_amd import dist as odist
    frames_total = 100_000_000 // 2
    a, b = odist.shard_range(frames_total, 3, 8)
    assert b - a == 6_250_000
    cfg = pkg.make_cfg()
    whole = engine.symbol_sweep(cfg, SNR, b - a, first_frame=a)
    m = (a + b) // 2
    halves = engine.symbol_sweep(cfg, SNR, m - a, first_frame=a) + engine.symbol_sweep(cfg, SNR, b - m, first_frame=m)
    assert np.array_equal(whole, halves)
    assert np.all(whole[:, 0] == b - a) and np.all(whole[:, 2] == 192 * (b - a))
    # a different chunking of the same range
    assert np.array_equal(whole, engine.symbol_sweep(cfg, SNR, b - a, first_frame=a, chunk_frames=1_000_003))


def test_c5_rank_shard_equals_halves(engine, pkg):
    """C5: 1e9 symbol-SNR evaluations on 8 GPUs -> 3.90625e6 frames per rank (4-tap Rayleigh, real AWGN, LS:
    the packed receiver with the channel on its clean spectra)."""
    from ofdm_amd import dist as odist
    frames_total = 1_000_000_000 // 16 // 2
    a, b = odist.shard_range(frames_total, 5, 8)
    cfg = pkg.make_cfg(noise="real", channel="rayleigh4")
    whole = engine.symbol_sweep(cfg, SNR, b - a, first_frame=a)
    m = a + 1_234_567
    halves = engine.symbol_sweep(cfg, SNR, m - a, first_frame=a) + engine.symbol_sweep(cfg, SNR, b - m, first_frame=m)
    assert np.array_equal(whole, halves)
    ber = whole[:, 3] / whole[:, 2]
    assert np.all(np.diff(ber[:8]) < 0)                 # BER falls with SNR (diversity-limited slope)


@pytest.mark.parametrize("workload", ["c4", "c5"])
def test_full_job_over_fake_ranks_equals_single_range(engine, pkg, workload):
    """SURVEY §4 "fake 8 ranks": the WHOLE job of C4 (1e8 symbols/point = 5e7 frames, AWGN + LS) and of C5
    (1e9 symbol-SNR evaluations = 3.125e7 frames, 4-tap Rayleigh + LS/ZF) split as dist.shard_range does
    for 2, 4 and 8 ranks, the shards run one after another on this device and summed on the host: every
    split equals the single-range sweep bit for bit (the sharded trial loop, /root/reference/src/OFDM.c:
    1195-1222; the counters are integer sums of per-frame terms)."""
    from ofdm_amd import dist as odist
    frames_total = 100_000_000 // 2 if workload == "c4" else 1_000_000_000 // 16 // 2
    cfg = pkg.make_cfg() if workload == "c4" else pkg.make_cfg(noise="real", channel="rayleigh4")
    whole = engine.symbol_sweep(cfg, SNR, frames_total)
    assert np.all(whole[:, 0] == frames_total) and np.all(whole[:, 2] == 192 * frames_total)
    for world in (8, 4, 2):
        parts = [engine.symbol_sweep(cfg, SNR, b - a, first_frame=a)
                 for a, b in (odist.shard_range(frames_total, r, world) for r in range(world))]
        assert np.array_equal(sum(parts), whole), world
        assert all(not np.array_equal(p, parts[0]) for p in parts[1:])      # the shards are distinct streams


def _sweep_worker(rank, world, port, n, out_path):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", OFDM_DIST_BACKEND="gloo")
    import ofdm_pkg
    pkg = ofdm_pkg.load()
    from ofdm_amd import dist as odist
    assert odist.init_from_env()
    import torch.distributed as dist
    with pkg.Engine(0) as eng:
        a, b = odist.shard_range(n, rank, world)
        c = eng.symbol_sweep(pkg.make_cfg(), SNR, b - a, first_frame=a)
    c = odist.allreduce_counters_np(c)
    if rank == 0:
        np.save(out_path, c)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_hip_symbol_sweep_equals_single(engine, pkg, tmp_path):
    n = 300_001
    out = tmp_path / "c.npy"
    mp.spawn(_sweep_worker, args=(2, _free_port(), n, str(out)), nprocs=2, join=True)
    got = np.load(out)
    assert np.array_equal(got, engine.symbol_sweep(pkg.make_cfg(), SNR, n))


def _main_worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", OFDM_DIST_BACKEND="gloo")
    import ofdm_pkg
    ofdm_pkg.load()
    from ofdm_amd import sweep
    import torch.distributed as dist
    sweep.reference_main(out_dir, trials=5001, snr_db=[6.0, 8.0, 10.0, 20.0])
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_reference_main_equals_single(pkg, tmp_path):
    """reference_main under torchrun forms the group itself and rank 0 writes the reduced
    files -- identical to the single-process files (frame mode: trials split by counter range)."""
    from ofdm_amd import sweep
    d2, d1 = tmp_path / "two", tmp_path / "one"
    d2.mkdir(); d1.mkdir()
    mp.spawn(_main_worker, args=(2, _free_port(), str(d2)), nprocs=2, join=True)
    sweep.reference_main(d1, trials=5001, snr_db=[6.0, 8.0, 10.0, 20.0])
    for name in ("Output_SNR.txt", "Output_EVM_AGC.txt", "Output_EVM_AGC_DB.txt", "Output_BER.txt"):
        assert (d2 / name).read_text() == (d1 / name).read_text(), name
    c2 = json.loads((d2 / "ofdm_sweep.json").read_text())
    c1 = json.loads((d1 / "ofdm_sweep.json").read_text())
    assert c2["counters"] == c1["counters"] and c2["world"] == 2


@pytest.mark.parametrize("workload,symbols", [("c3", 200_000), ("c4", 400_000)])
def test_torchrun_bench_rccl(workload, symbols):
    """bench.py under torch.distributed.run (one rank): init_process_group("nccl") + the RCCL
    all-reduce of the counters execute on the GPU; the JSON line is well formed."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py"), "--gpus", "1",
           "--workload", workload, "--symbols", str(symbols), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert "RCCL all-reduce" in line["config"]["parallelism"]
    assert line["results"]["frames_per_snr"] == symbols // 2
    assert line["scaling"] == ("weak" if workload == "c3" else "strong")


@pytest.mark.parametrize("workload,symbols,frames_per_snr",
                         [("c3", 200_000, 2 * 100_000),     # weak: each rank its own 100,000 frames
                          ("c4", 400_000, 200_000),         # strong: 200,000 frames in total, split over 2 ranks
                          ("fft64", 1 << 16, None)])
def test_bench_gpus2_self_launch_gloo(workload, symbols, frames_per_snr):
    """`bench.py --gpus 2` outside torchrun launches its own 2 ranks (torch.distributed.run as a
    child) and relays rank 0's line.  On this 1-GPU box the ranks share cuda:0 and reduce over gloo
    (OFDM_DIST_BACKEND=gloo; RCCL refuses two ranks on one GPU): the weak/strong range split, the per-step
    counter all-reduce, the max-over-ranks time and the whole-job value run at world 2 (the sharded trial loop,
    /root/reference/src/OFDM.c:1195-1222)."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", workload, "--symbols", str(symbols),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, PYTHONUNBUFFERED="1", OFDM_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout.strip().splitlines()
    assert len(out) == 1, out
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["parallelism"].startswith("dp2") and line["config"]["backend"] == "gloo"
    if frames_per_snr is None:
        # weak: both ranks' 2 launches x 2^16 transforms per step
        assert line["value"] == pytest.approx(2 * 2 * symbols * line["steps"] / (line["ms_per_step"] * line["steps"] / 1e3))
        assert line["results"]["fft_ifft_roundtrip_max_rel_err"] < 1e-5
        return
    assert line["results"]["frames_per_snr"] == frames_per_snr
    per_gpu = symbols // 2 if workload == "c3" else symbols // 2 // 2
    assert line["config"]["frames_per_gpu"] == per_gpu
    units = frames_per_snr * 2 * 16 * line["steps"]
    assert line["value"] == pytest.approx(units / (line["ms_per_step"] * line["steps"] / 1e3))
