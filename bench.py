#!/usr/bin/env python3
"""Benchmark: OFDM symbols/sec over the BER-vs-SNR sweep on MI355X (BASELINE.json metric).

One step = one full sweep of the hot path over one batch: the Tx pass (K2, data symbols written to
HBM once, OFDM.c:1191) and the per-SNR over-the-air + receive pass (K3, 16 SNR points 0..30 dB,
OFDM.c:1202-1211) for every frame, then ONE all-reduce of the int64 counters.  Inputs (the Tx
batch) live in HBM for the whole step.  Workload (default, --workload c3 = BASELINE configs[2]):
802.11a 64-subcarrier QPSK, real AWGN (D7), LTF least-squares estimate + ZF + slicer + EVM,
1e7 data symbols per SNR point per GPU (weak scaling).  `value` = data OFDM symbols received and
scored per second over the whole job (symbols x SNR points / wall).

Launched as `python bench.py --gpus N --steps K --warmup W`, or for N > 1 under
`torch.distributed.run` (one rank per GPU, RCCL all-reduce).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import ofdm_pkg  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_SYMBOL_SNR = 652     # 80 x 8 B clean symbol + 12 B packed truth bits

WORKLOADS = {
    # name: (config description, cfg kwargs, symbols per SNR point per GPU, snr grid)
    "c3": ("BASELINE configs[2]: AWGN sweep 0-30 dB step 2 + LTF LS channel est + slicer/EVM, 1e7 symbols/point",
           dict(est="ls", noise="real", channel="awgn", conv="c", payload="random"), 10_000_000),
    "c2": ("BASELINE configs[1]: AWGN BER sweep 0-30 dB step 2, ideal channel, 1e6 symbols/point",
           dict(est="ideal", noise="real", channel="awgn", conv="c", payload="random"), 1_000_000),
    "c5": ("BASELINE configs[4] per-GPU shard: 4-tap Rayleigh + ZF, LS estimate, complex AWGN",
           dict(est="ls", noise="complex", channel="rayleigh4", conv="c", payload="random", kappa=1.0),
           10_000_000),
    # the reference's own trial (OFDM.c main loop): capture + packet detection/selection + CFO + LS
    # + demap, 2 data symbols per trial -- the like-for-like line next to cpu_baseline
    "frame": ("frame mode: OFDM.c Transmission_Over_Air + Receiver trials (sync, CFO, LS), reference message",
              dict(payload="message", noise="real", conv="c"), 1_000_000),
}
FRAME_CAPTURE_BYTES = 3008 * 8     # capture samples read per trial (L2-resident 78 KB waveform)
SNR_GRID = np.arange(0.0, 31.0, 2.0)


VALU_PEAK_PER_S = 256 * 4 * 0.5 * 2.4e9   # wave64 VALU instructions/s: 1 per 2 cycles per SIMD (tools/ubench_valu.hip)


def load_pmc(workload: str) -> dict:
    """Per-launch rocprofv3 --pmc figures for this workload (profiles/pmc_summary.json, written by
    tools/pmc_summary.py from tools/gpu_profile.sh runs), or {}."""
    p = ROOT / "profiles" / "pmc_summary.json"
    try:
        return json.loads(p.read_text()).get(workload, {})
    except Exception:
        return {}


def _ref_worker(args):
    """One host process running the reference's own trial loop (spawned: no GPU state)."""
    snr, n, seed = args
    from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
    t, acc = RefLib().time_trials(snr, n, seed)
    return n, t, float(acc[2])


def host_cores() -> int:
    """Host cores this process may use, capped at the GPU box's per-GPU CPU share (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(seconds: float = 12.0) -> dict | None:
    """The reference itself (oracle/_ref/libofdm_ref.so, the unmodified OFDM.c built with gcc -O2)
    timed on this host: its own trial loop (Transmission_Over_Air + Receiver, 2 data symbols per
    trial) at 10 dB -- BASELINE configs[0].  The reference is single-threaded with global state, so
    the node figure runs one process per host core (up to the box's 16-core share), each ~`seconds`
    of trials; the one-thread figure is reported beside it.  Runs before the GPU is initialised."""
    import multiprocessing as mp
    try:
        from oracle import RefLib, Oracle  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
        ref = RefLib()
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "OFDM symbols/s", "cores": 0, "kind": "reference",
                "sample": f"unavailable: {e}"}
    cpu = platform.processor() or platform.machine()
    t, _ = ref.time_trials(10.0, 50, 1)            # calibrate
    per_trial = max(t / 50, 1e-6)
    n1 = max(100, int(seconds / 2 / per_trial))
    t1, acc1 = ref.time_trials(10.0, n1, 7)
    single = {"value": 2 * n1 / t1, "unit": "OFDM symbols/s", "cores": 1, "kind": "reference",
              "sample": f"{n1} reference trials on 1 thread in {t1:.1f} s; mean BER {acc1[2] / n1:.3g}"}
    P = host_cores()
    n = max(100, int(seconds / per_trial))
    jobs = [(10.0, n, 1000 + k) for k in range(P)]
    with mp.get_context("spawn").Pool(P) as pool:
        w0 = time.perf_counter()
        res = pool.map(_ref_worker, jobs, chunksize=1)
        wall = time.perf_counter() - w0
    trials = sum(r[0] for r in res)
    out = {"value": 2 * trials / wall, "unit": "OFDM symbols/s", "cores": P, "kind": "reference",
           "sample": f"{trials} reference trials (Transmission_Over_Air + Receiver of src/OFDM.c, gcc -O2, "
                     f"frame mode, 2 data symbols each) at SNR 10 dB in {wall:.1f} s wall on {P} host "
                     f"processes of {cpu} ({os.cpu_count()} CPUs visible); mean BER "
                     f"{sum(r[2] for r in res) / trials:.3g}",
           "single_core": single}
    try:   # our CPU restatement of the GPU workload's symbol chain, for scale (port, 1 thread)
        O = Oracle()
        nf = 2000
        tt, _ = O.time_symbol_sweep(O.cfg(), SNR_GRID, nf)
        out["port_symbol_chain"] = {"value": 2 * nf * len(SNR_GRID) / tt, "unit": "OFDM symbols/s", "cores": 1,
                                    "kind": "port", "sample": f"{nf} frames x {len(SNR_GRID)} SNR of the c3 chain"}
    except Exception:
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--symbols", type=int, default=0, help="override data symbols per SNR point per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    rank0_single = int(os.environ.get("RANK", "0")) == 0 and int(os.environ.get("WORLD_SIZE", "1")) == 1
    # host-side reference timing first, before anything touches the GPU (worker processes are spawned)
    cpu = cpu_baseline(args.cpu_seconds) if rank0_single and not args.no_cpu_baseline else None

    import torch
    import torch.distributed as dist
    pkg = ofdm_pkg.load()
    from ofdm_amd import abi, dist as odist

    rank, world, local = odist.env_rank_world()
    # under torch.distributed.run (RANK set) the RCCL group is formed even for one rank
    distributed = world > 1 or "RANK" in os.environ
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = local if distributed else 0

    desc, kw, symbols = WORKLOADS[args.workload]
    if args.symbols:
        symbols = args.symbols
    frames = symbols // 2                       # D = 2 data symbols per frame
    cfg = pkg.make_cfg(**kw)
    eng = pkg.Engine(dev)
    first, _ = odist.weak_range(frames, rank)
    frame_mode = args.workload == "frame"
    counters = eng.new_counters(len(SNR_GRID))
    if not frame_mode:
        tx, bits = eng.tx_buffers(frames)

    def step():
        if frame_mode:            # one trial = one frame of 2 data symbols; waveform cached on the device
            c = eng.frame_sweep(cfg, SNR_GRID, frames, first_trial=first)
            counters.copy_(torch.from_numpy(c))
        else:
            counters.zero_()
            eng.tx_frames(cfg, first, frames, tx, bits)
            eng.rx_frames(cfg, tx, bits, first, frames, SNR_GRID, counters)
        odist.allreduce_counters(counters)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.timing(True)
    eng.timing_reset()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.timing(False)
    rx_ms, rx_n = eng.timing_query(abi.K_FRAME if frame_mode else abi.K_RX)
    tx_ms, tx_n = eng.timing_query(abi.K_TX)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    c = counters.cpu().numpy()
    n_snr = len(SNR_GRID)
    total_units = float(world) * frames * 2 * n_snr * args.steps     # symbol-SNR evaluations
    value = total_units / elapsed
    rx_avg_s = rx_ms / max(rx_n, 1) / 1e3
    units_per_launch = frames * 2 * n_snr                            # one launch covers all 16 SNR points
    bytes_per_unit = FRAME_CAPTURE_BYTES / 2 if frame_mode else BYTES_PER_SYMBOL_SNR
    achieved = units_per_launch * bytes_per_unit / rx_avg_s / 1e9
    res = pkg.SweepResult(SNR_GRID, c)
    pmc = load_pmc(args.workload)
    if rank == 0:
        line = {
            "metric": "OFDM symbols/sec (whole node) over BER-vs-SNR sweep; achieved HBM GB/s vs peak",
            "value": value,
            "unit": "OFDM symbols/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox4x32-10 bits and noise, seed 0x80211A)",
            "config": {"workload": args.workload, "description": desc, "symbols_per_snr_per_gpu": 2 * frames,
                       "snr_db": SNR_GRID.tolist(), "frames_per_gpu": frames, "data_symbols_per_frame": 2,
                       "parallelism": f"dp{world} (counter-range shards, 1 RCCL all-reduce)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc.get("rx_hbm_bytes_per_launch"),
                         "kernel": "frame_sync_kernel+frame_sym_kernel" if frame_mode
                                   else ("rx_ls_kernel" if kw.get("est") == "ls" else "rx_ideal_kernel"),
                         "bytes_per_unit": bytes_per_unit,
                         "units_per_launch": units_per_launch,
                         "avg_launch_ms": rx_avg_s * 1e3, "launches": rx_n,
                         "traffic_note": "HBM bytes per launch from FETCH_SIZE x2 (gfx950) + WRITE_SIZE, "
                                         "profiles/pmc_summary.json; each symbol is staged once per launch "
                                         "and re-used from LDS for every SNR point"},
            # the kernel is VALU-issue bound: measured VALU wave-instructions per unit
            # (SQ_INSTS_VALU / units, rocprofv3) x units / live launch time vs the issue peak
            "valu_roofline": ({"achieved": units_per_launch * pmc["valu_instr_per_unit"] / rx_avg_s,
                               "peak": VALU_PEAK_PER_S, "unit": "wave-instr/s",
                               "frac": units_per_launch * pmc["valu_instr_per_unit"] / rx_avg_s / VALU_PEAK_PER_S,
                               "instr_per_unit": pmc["valu_instr_per_unit"]}
                              if pmc.get("valu_instr_per_unit") else None),
            "kernels_ms": {"rx_total": rx_ms, "rx_launches": rx_n, "tx_total": tx_ms, "tx_launches": tx_n},
            "results": {"ber": res.ber.tolist(), "evm_pre_db": res.evm_pre_db.tolist()},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    eng.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
