#!/usr/bin/env python3
"""Path rates of frame_sync_long_kernel on bench.py's frame8 workload (TEST INFRASTRUCTURE: uses the oracle's
waveform; tools/frame8_mix.py reads the fixture to weight the kernel's blocks).

Per SNR point of the bench grid, over captures of the 8-symbol bench message's waveform (oracle.frame_waveform,
the same bits as the GPU's ofdm_set_message) with real-only AWGN at sigma^2 = P_wave / 10^(snr / 10) (the GPU's
frame-mode noise, ofdm_frame.hip): Packet_Detection's M (OFDM.c:659-683, tests/test_lazy_rule.corr_out) and the
kernel's decisions --
  decided   rounds 0-1 (positions [0, 2 x 1,984)) decide Packet_Selection (the lazy round-2 skip);
  regen     the matched filter's window [p + 140, p + 2 (nfr - 1) + 10] (the samples its runs read: the first instant
            read is frame sample 80) is not all in the capture ring after the last detection round's piece
            (ofdm_frame.hip, the long kernel's residency rule: the ring holds the last LW_RING - 3 = 2,973 samples
            generated, [1,042, 4,015) for decided items, [L - 2,973, L) for undecided ones), so its missing end is
            generated: regen_full = its whole passes (4 Philox blocks per lane, 256 per pass) per item, regen_tail3 /
            2 / 1 = the fraction of items whose last pass draws 3 / 2 / 1 blocks per lane (ceil(rest / 64)), and
            regen_passes = the passes counted as whole ones (the pre-trim cost, for comparison); regen_fwd: the items
            whose window's END is generated (past the ring)
  sync_fail no packet selected (p = 0).
The rates are statistical (double precision here, fp32 sums on the GPU: a capture at the 0.75 threshold may fall
either way), so the fixture carries its sample size.

usage: python tests/golden/gen_frame8_rates.py [--captures 600]   ->  tests/golden/frame8_path_rates.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

LW_ROUND = 64 * 31
LW_RING = 2976
LEN_RRC_RX = 10
SNR_GRID = np.arange(0.0, 31.0, 2.0)


def selection(m: np.ndarray, limit: int):
    """the kernels' Packet_Selection over positions below `limit` (OFDM.c:685-771): (decided, packet_idx); packet_idx
    0 when no front qualifies"""
    idx = np.nonzero(m[:limit] > 0.75)[0]
    if len(idx) == 0:
        return False, 0
    prev = np.concatenate([[-1], idx[:-1]])
    fronts = idx[(idx - prev) > 300]
    valid = [f for f in fronts if f + 230 < limit and m[f + 230] > 0.75]
    if not valid or valid[0] >= fronts.max():
        return False, 0
    return True, int(valid[0]) + LEN_RRC_RX + 1


def rates(wave: np.ndarray, snr_db: float, n: int, seed: int) -> dict:
    from test_lazy_rule import corr_out  # noqa: PLC0415
    L = int(0.307 * len(wave))
    Lc = L - 47
    nfr = 320 + 80 * 8
    sigma = np.sqrt(np.mean(np.abs(wave) ** 2) / 10 ** (snr_db / 10))
    rng = np.random.default_rng(seed)
    dec = regen = fail = passes = nf = full = 0
    tails = {1: 0, 2: 0, 3: 0}
    for _ in range(n):
        s = int(rng.integers(0, len(wave) - L))
        cap = wave[s:s + L] + sigma * rng.standard_normal(L)       # real-only AWGN (D7)
        m = corr_out(cap)
        d, p = selection(m, min(2 * LW_ROUND, Lc))
        if not d:
            ok, p = selection(m, Lc)
            p = p if ok else 0
        lo, hi = p + 2 * 80 - 20, min(p + 2 * (nfr - 1) + 10, L - 1)
        held = 1 if d else 2
        res_hi = min(L, held * LW_ROUND + LW_ROUND + 47)
        res_lo = res_hi + 3 - LW_RING
        dec += d
        if hi >= res_hi or lo < res_lo:
            fwd = hi >= res_hi                                      # the window's end is generated, else its start
            g0, g1 = (max(lo, res_hi), hi + 1) if fwd else (lo, min(hi + 1, res_lo))
            blocks = ((s + g1 - 1) >> 2) - ((s + g0) >> 2) + 1      # the capture start s is the kernel's rx_start
            if blocks > 0:
                regen += 1
                passes += -(-blocks // 256)
                nf += fwd
                # capture_blocks<..., TRIM>: whole passes while more than 192 blocks remain, then one of 3 / 2 / 1
                f = 0
                while blocks > 192:
                    f, blocks = f + 1, blocks - 256
                if blocks > 128:
                    tails[3] += 1
                elif blocks > 64:
                    tails[2] += 1
                elif blocks > 0:
                    tails[1] += 1
                full += f
        fail += p == 0
    return {"snr_db": snr_db, "captures": n, "decided": dec / n, "regen": regen / n, "regen_passes": passes / n,
            "regen_full": full / n, "regen_tail3": tails[3] / n, "regen_tail2": tails[2] / n,
            "regen_tail1": tails[1] / n, "regen_fwd": nf / n, "sync_fail": fail / n}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--captures", type=int, default=600)
    a = ap.parse_args(argv)
    from oracle import Oracle  # noqa: PLC0415
    import importlib.util  # noqa: PLC0415
    spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    O = Oracle()
    wave = O.frame_waveform(O.message_bits(bench.FRAME8_MESSAGE)).astype(np.complex128)
    rows = [rates(wave, float(s), a.captures, 1000 + k) for k, s in enumerate(SNR_GRID)]
    out = {"generator": f"tests/golden/gen_frame8_rates.py --captures {a.captures}",
           "message": bench.FRAME8_MESSAGE.decode(), "capture_len": int(0.307 * len(wave)),
           "rows": rows,
           "grid_mean": {k: float(np.mean([r[k] for r in rows])) for k in (
               "decided", "regen", "regen_passes", "regen_full", "regen_tail3", "regen_tail2", "regen_tail1", "regen_fwd",
               "sync_fail")}}
    (HERE / "frame8_path_rates.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out["grid_mean"]))


if __name__ == "__main__":
    main()
