"""The reference's main() (src/OFDM.c:1187-1236) on the MI355X engine.

reference_main() sweeps SNR 6..40 dB step 1 (OFDM.c:18, 1195-1198) and writes the same four
files into out_dir (data/ by default): Output_SNR.txt, Output_EVM_AGC.txt (EVM before the slicer),
Output_EVM_AGC_DB.txt (EVM after the slicer) and Output_BER.txt, so scripts/OFDM_Plotting.py
runs unchanged.  The reference runs ONE trial per SNR point (frame mode, fixed message); here
`trials` is a parameter and the per-point values are pooled over them (BER = errors / bits,
EVM = 10 log10(sum|e|^2 / sum|d|^2)); with trials=1 they equal the reference's per-trial values.
`mode="symbol"` runs the per-symbol chain (genie timing, LTF LS estimate) instead.

Per-point values in the files.  Output_EVM_AGC.txt / Output_EVM_AGC_DB.txt hold, for trials > 1,
the MEAN over trials of the per-trial EVM_dB the reference writes for its one trial
(OFDM.c:1126,1150); the post-slicer mean is -inf as soon as one trial had no slicer error, as the
reference's own value for that trial is (ref_mc_curve.json's mean_evm_agc_db is the same
statistic).  evm="finite" keeps that pre-slicer file and writes, after the slicer, the mean over the trials
whose value is finite (trials with >= 1 slicer error; their count goes to the sidecar), so a many-trial
run stays plottable above ~3 dB.  evm="pooled" writes 10 log10(sum|e|^2 / sum|d|^2) over all trials
instead.  BER is errors / bits (= the mean per-trial BER: every trial carries the same bit count).

Multi-GPU: launched under torchrun, each rank takes a contiguous share of the trials
(dist.shard_range); reference_main() forms the process group (dist.init_from_env: RCCL, or gloo
with OFDM_DIST_BACKEND=gloo) and the counters are summed with one all-reduce before rank 0 writes.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

from . import abi, dist
from .engine import Engine, SweepResult
from .fileio import write_reference_outputs

REF_SNR = np.arange(6.0, 41.0, 1.0)        # OFDM.c:18, 1197


def run_sweep(engine: Engine, snr_db, trials: int, mode: str = "frame", seed: int = 0x80211A,
              payload: str | None = None, est: str = "ls", noise: str = "real", channel: str = "awgn",
              conv: str = "c", rank: int = 0, world: int = 1, message: str | None = None) -> SweepResult:
    snr = np.asarray(snr_db, np.float64)
    if message is not None:
        engine.set_message(message)             # OFDM.c:20 `message`, framed by Data_Generator
    start, end = dist.shard_range(trials, rank, world)
    if mode == "frame":
        cfg = abi.make_cfg(seed=seed, conv=conv, payload=payload or "message", noise=noise)
        c = engine.frame_sweep(cfg, snr, end - start, first_trial=start, mode="c" if conv == "c" else "matlab")
    elif mode == "symbol":
        cfg = abi.make_cfg(seed=seed, conv=conv, payload=payload or "random", est=est, noise=noise, channel=channel)
        c = engine.symbol_sweep(cfg, snr, end - start, first_frame=start)
    else:
        raise ValueError(mode)
    if world > 1:
        c = dist.allreduce_counters_np(c, engine.device)
    return SweepResult(snr, c)


def reference_main(out_dir: str | Path = "data", trials: int = 1, mode: str = "frame", snr_db=REF_SNR,
                   seed: int = 0x80211A, device: int = 0, json_sidecar: bool = True, evm: str = "trial",
                   **kw) -> SweepResult:
    if evm not in ("trial", "finite", "pooled"):
        raise ValueError(evm)
    rank, world, local = dist.env_rank_world()
    if world > 1:
        dist.init_from_env()
    t0 = time.perf_counter()
    with Engine(local if world > 1 else device) as eng:
        res = run_sweep(eng, snr_db, trials, mode=mode, seed=seed, rank=rank, world=world, **kw)
    wall = time.perf_counter() - t0
    if rank == 0:
        pre, post = {"trial": (res.mean_frame_evm_db, res.mean_frame_evm_post_db),
                     "finite": (res.mean_frame_evm_db, res.mean_finite_frame_evm_post_db),
                     "pooled": (res.evm_pre_db, res.evm_post_db)}[evm]
        write_reference_outputs(out_dir, res.snr_db, pre, post, res.ber)
        if json_sidecar:
            side = {"mode": mode, "trials_per_snr": trials, "world": world, "seed": seed, "wall_s": wall,
                    "evm_files": evm, "snr_db": res.snr_db.tolist(), "ber": res.ber.tolist(),
                    "mean_trial_evm_db": res.mean_frame_evm_db.tolist(),
                    "mean_trial_evm_post_db": [float(v) for v in res.mean_frame_evm_post_db],
                    "mean_finite_trial_evm_post_db": [float(v) for v in res.mean_finite_frame_evm_post_db],
                    "post_finite_trials": res.counters[:, abi.C_EVMDB_POST_FINITE].tolist(),
                    "evm_pre_db": res.evm_pre_db.tolist(),
                    "evm_post_db": [float(v) for v in res.evm_post_db], "sync_fail_rate": res.sync_fail_rate.tolist(),
                    "counters": res.counters.tolist()}
            (Path(out_dir) / "ofdm_sweep.json").write_text(json.dumps(side, indent=1))
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description="802.11a OFDM-QPSK Monte-Carlo sweep on MI355X (OFDM.c main())")
    ap.add_argument("--out", default="data")
    ap.add_argument("--trials", type=int, default=1, help="trials (frame mode) or frames (symbol mode) per SNR")
    ap.add_argument("--mode", choices=["frame", "symbol"], default="frame")
    ap.add_argument("--snr", type=float, nargs="*", help="SNR grid in dB (default 6..40 step 1)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x80211A)
    ap.add_argument("--est", choices=["ls", "ideal"], default="ls")
    ap.add_argument("--noise", choices=["real", "complex", "none"], default="real")
    ap.add_argument("--channel", choices=["awgn", "rayleigh4"], default="awgn")
    ap.add_argument("--conv", choices=["c", "matlab"], default="c")
    ap.add_argument("--payload", choices=["random", "message", "tester"])
    ap.add_argument("--message", help="MESSAGE payload text (default: OFDM.c:20), up to 96 characters")
    ap.add_argument("--evm", choices=["trial", "finite", "pooled"], default="trial",
                    help="EVM files: mean of per-trial EVM_dB (the reference's statistic, -inf after the slicer "
                         "once one trial is clean), the same with the post-slicer mean over finite trials, or pooled")
    ap.add_argument("--print-messages", action="store_true",
                    help="as OFDM.c:1167-1182: receive one capture per SNR point and print the decoded text")
    a = ap.parse_args(argv)
    snr = np.array(a.snr) if a.snr else REF_SNR
    res = reference_main(a.out, a.trials, a.mode, snr, a.seed, est=a.est, noise=a.noise, channel=a.channel,
                         conv=a.conv, payload=a.payload, message=a.message, evm=a.evm)
    for s, b, e in zip(res.snr_db, res.ber, res.evm_pre_db):
        print(f"SNR = {s:5.1f} dB   BER = {b:.3e}   EVM = {e:7.2f} dB", file=sys.stderr)
    if a.print_messages:
        for line in received_messages(snr, a.message, a.seed):
            print(line)


def received_messages(snr_db, message: str | None = None, seed: int = 0x80211A, device: int = 0):
    """One reference trial per SNR point -- Transmission_Over_Air + capture + Receiver (OFDM.c:1202-1211)
    -- yielding the console text the reference prints (OFDM.c:1177-1181)."""
    with Engine(device) as eng:
        if message is not None:
            eng.set_message(message)
        nd = eng.payload_frames("message")
        w = eng.transmitter("c", "message")
        L = abi.capture_len(nd)
        rng = np.random.default_rng(seed)
        for i, s in enumerate(np.asarray(snr_db, np.float64)):
            ota = eng.transmission_over_air(w, float(s), seed=seed, trial=0, snr_index=i)
            rs = int(rng.integers(0, len(w) - L))               # rand() % (len - cap) (OFDM.c:949)
            o = eng.receiver(ota[rs:rs + L], "c", "message")
            yield f"SNR = {s:.0f} dB\nReceived Message: \n{o['message']}"


if __name__ == "__main__":
    main()
