#!/usr/bin/env python3
"""Generate the committed golden fixtures from the COMPILED REFERENCE (oracle/_ref, built from the
unmodified /root/reference/src/OFDM.c) and from the reference's own data files.

Run in the build container (the GPU box has no /root/reference):
    python tests/golden/gen_golden.py [--only mc] [--mc-trials 48000 --mc-deep-trials 1000000]

Outputs (all plain data, loadable with numpy allow_pickle=False / json):
  fft_vectors.npz      200 random 64-pt inputs and the reference's fft()/ifft() outputs (OFDM.c:314-339)
  tx_waveform.npz      Transmitter() output (9800 cf32), Data bits, Data_Payload_Mod, Long_preamble_slot_Frequency,
                       RRC taps (OFDM.c:20-34, 467-618)
  rx_stages.npz        Receiver() intermediates for injected-noise captures (OFDM.c:941-1165)
  matlab_output.npz    the 96 KAT bits of data/Matlab_Output.txt (MATLAB Tester RX_Payload_1_demod)
  reference_data.json  the four data/Output_*.txt files of the reference run (format fixtures)
  ref_mc_curve.json    Monte-Carlo BER/EVM of the reference's own trial loop (TOA+Receiver) per SNR
  ref_genie_ls_curve.json  genie-timed symbol chain built from the reference's own ifft/fft/
                       Channel_Estimation (two separately noised LTF windows), real noise
                       sigma^2 = 0.4980 * 52/4096 / snr: pins symbol mode's LS estimator statistically
  ref_symbol_chain_curve.json  the same chain entirely from the reference's stage functions and its
                       gaussian_noise, 0..30 dB step 2, 2e6 frames at 8 / 10 dB and 1e7 at 12 dB (>= 1,000 bit
                       errors each) with per-frame error statistics (frame-clustered BER variance)
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
from oracle import RefLib, build_ref  # noqa: E402

REF_DATA = Path("/root/reference/data")


def gen_fft(R: RefLib):
    rng = np.random.default_rng(802111)
    x = (rng.standard_normal((200, 64)) + 1j * rng.standard_normal((200, 64))).astype(np.complex64)
    # include structured vectors: impulses, constants, OFDM-like sparse spectra
    x[0] = 0; x[0, 0] = 1
    x[1] = 0; x[1, 17] = 1 - 2j
    x[2] = 1
    f = np.stack([R.fft(v) for v in x])
    i = np.stack([R.ifft(v) for v in x])
    np.savez_compressed(HERE / "fft_vectors.npz", x=x, fft=f, ifft=i)


def gen_tx(R: RefLib):
    g = R.globals()
    np.savez_compressed(HERE / "tx_waveform.npz", waveform=R.waveform(), bits=g["bits"],
                        payload_mod=g["payload_mod"], ltf_freq=g["ltf_freq"], dims=g["dims"],
                        rrc_taps=R.rrc_taps())


def gen_rx(R: RefLib):
    w = R.waveform()
    P = float(np.mean(np.abs(w.astype(np.complex128)) ** 2))
    cases = [(30.0, 0, 11), (20.0, 1234, 12), (14.0, 777, 13), (10.0, 3000, 14), (8.0, 50, 15),
             (6.0, 6000, 16), (12.0, 4321, 17), (100.0, 0, 18)]
    out = {"snr": [], "rx_start": [], "noise": [], "packet_idx": [], "corr": [], "rxframe": [],
           "coarse": [], "fine": [], "H": [], "Yf": [], "nopilot": [], "bits": [], "res": [], "res_receiver": []}
    for snr, rs, seed in cases:
        rng = np.random.default_rng(seed)
        sigma = np.sqrt(P / 10 ** (snr / 10))
        # injected real-only noise (D7) on the captured window only
        noise = np.zeros(len(w), np.float32)
        noise[rs:rs + 3008] = (sigma * rng.standard_normal(3008)).astype(np.float32)
        ota = (w + noise).astype(np.complex64)
        d = R.receiver_stages(ota, rs)
        rr = R.receiver(ota, rs)
        assert np.array_equal(np.nan_to_num(rr, neginf=-999), np.nan_to_num(d["res"], neginf=-999)), (rr, d["res"])
        out["snr"].append(snr); out["rx_start"].append(rs); out["noise"].append(noise[rs:rs + 3008])
        out["packet_idx"].append(d["packet_idx"]); out["res_receiver"].append(rr)
        for k in ("corr", "rxframe", "coarse", "fine", "H", "Yf", "nopilot", "bits", "res"):
            out[k].append(d[k])
    np.savez_compressed(HERE / "rx_stages.npz", **{k: np.array(v) for k, v in out.items()})


def gen_kat():
    kat = np.array([int(float(t)) for t in (REF_DATA / "Matlab_Output.txt").read_text().split()], np.int32)
    np.savez_compressed(HERE / "matlab_output.npz", bits=kat)
    files = {n: (REF_DATA / n).read_text() for n in
             ("Output_SNR.txt", "Output_EVM_AGC.txt", "Output_EVM_AGC_DB.txt", "Output_BER.txt")}
    (HERE / "reference_data.json").write_text(json.dumps(files, indent=1))


# fftshifted data bins / pilots of the subcarrier map (OFDM.c:523-548)
DATA_IDX = np.array([*range(6, 11), *range(12, 25), *range(26, 32), *range(33, 39), *range(40, 53), *range(54, 59)])
PILOTS = {11: 1.0, 25: 1.0, 39: 1.0, 53: -1.0}


def gen_genie(R: RefLib, frames: int = 20000, snrs=(0.0, 2.0, 4.0, 6.0)):
    rng = np.random.default_rng(80211)
    T = R.ifft(R.globals()["ltf_freq"])                       # long training symbol, C ifft (D5)
    ltf160 = np.concatenate([T[32:], T, T])
    s2 = 1 / np.sqrt(2)
    rows = []
    for snr in snrs:
        sigma = np.sqrt(0.4980 * 52 / 4096 / 10 ** (snr / 10))
        nbits = nerr = 0
        epre = 0.0
        for _ in range(frames):
            frame = np.zeros(480, np.complex64)
            frame[160:320] = ltf160
            bits = rng.integers(0, 2, (2, 96))
            for d in range(2):
                b0, b1 = bits[d, 0::2], bits[d, 1::2]
                # 00:(1+j) 01:(-1+j) 10:(-1-j) 11:(1-j), /sqrt2 (OFDM.c:423-430)
                q = (np.where(b0 == b1, 1.0, -1.0) + 1j * np.where(b0 == 1, -1.0, 1.0)) * s2
                X = np.zeros(64, np.complex64)
                X[DATA_IDX] = q
                for k, v in PILOTS.items():
                    X[k] = v
                x = R.ifft(X)
                frame[320 + 80 * d:400 + 80 * d] = np.concatenate([x[48:], x])
            rx = (frame + (sigma * rng.standard_normal(480)).astype(np.float32)).astype(np.complex64)  # D7
            H = R.channel_estimation(rx)
            for d in range(2):
                Y = R.fft(rx[336 + 80 * d:400 + 80 * d])
                z = Y[DATA_IDX].astype(np.complex128) / H[DATA_IDX]
                pr, pi = z.real > 0, z.imag > 0
                c0, c1 = (~pi).astype(int), (pr != pi).astype(int)
                nerr += int(np.sum(c0 != bits[d, 0::2]) + np.sum(c1 != bits[d, 1::2]))
                nbits += 96
                b0, b1 = bits[d, 0::2], bits[d, 1::2]
                ref = (np.where(b0 == b1, 1.0, -1.0) + 1j * np.where(b0 == 1, -1.0, 1.0)) * s2
                epre += float(np.sum(np.abs(z - ref) ** 2))
        rows.append({"snr_db": snr, "frames": frames, "bits": nbits, "bit_err": nerr, "evm_terms": nbits // 2,
                     "sum_evm_pre": epre})
    meta = {"generator": "tests/golden/gen_golden.py gen_genie",
            "source": "reference ifft/fft/Channel_Estimation (OFDM.c:314-339, 830-850), numpy real noise",
            "rows": rows}
    (HERE / "ref_genie_ls_curve.json").write_text(json.dumps(meta, indent=1))


CHAIN_SNRS = [float(x) for x in range(0, 31, 2)]            # bench.py's SNR grid
CHAIN_FRAMES = 200_000                                     # per point: EVM to ~0.001 dB, BER down to 4 dB
CHAIN_DEEP = {8.0: 2_000_000, 10.0: 2_000_000, 12.0: 10_000_000}   # >= 1,000 bit errors each
CHAIN_JOB = 100_000                                        # frames per job, seeded by job index


def _chain_worker(args):
    snr, n, seed = args
    return snr, RefLib().symbol_chain_stats(snr, n, seed).tolist()


def chain_jobs(snrs=CHAIN_SNRS) -> list:
    jobs = []
    for snr in snrs:
        n = CHAIN_DEEP.get(snr, CHAIN_FRAMES)
        jobs += [(snr, CHAIN_JOB, 3000017 * (j + 1) + int(snr)) for j in range(n // CHAIN_JOB)]
    return jobs


def chain_rows(res: list) -> list:
    """fixture rows from (snr, acc5) job results, summed in job order"""
    acc = {}
    for snr, a in res:
        acc[snr] = [x + y for x, y in zip(acc.get(snr, [0.0] * 5), a)]
    rows = []
    for snr in sorted(acc):
        be, nb, epre, be2, fe = acc[snr]
        rows.append({"snr_db": snr, "frames": int(nb) // 192, "bits": int(nb), "bit_err": int(be),
                     "evm_terms": int(nb) // 2, "sum_evm_pre": epre, "sum_frame_err_sq": int(be2),
                     "frames_with_err": int(fe)})
    return rows


def gen_chain(procs: int):
    """ref_symbol_chain_curve.json: the genie symbol chain built from the reference's own stage functions
    (ref_harness.c ref_time_symbol_chain: QPSK_Modulator, ifft, gaussian_noise, Channel_Estimation, fft,
    AGC_Receiver, QPSK_Demodulator -- OFDM.c:415-433, 320-339, 622-655, 830-850, 314-318, 852-908) over the
    bench's SNR grid, with the per-frame error statistics that give the frame-clustered BER variance.
    Jobs of CHAIN_JOB frames seeded 3000017 (j + 1) + snr, so the file does not depend on --procs."""
    with mp.Pool(procs) as pool:
        res = pool.map(_chain_worker, chain_jobs(), chunksize=1)     # job order: sums independent of --procs
    rows = chain_rows(res)
    meta = {"generator": f"tests/golden/gen_golden.py --only chain (jobs of {CHAIN_JOB} frames)",
            "source": "reference OFDM.c stage functions (gcc -O2) composed as the genie symbol chain "
                      "(oracle/ref_harness.c ref_time_symbol_chain, flags 4), real noise "
                      "sigma^2 = 0.4980 * 52/4096 / 10^(snr/10), LCG rand hook",
            "seeds": "job j of a point: noise 3000017 (j + 1) + snr, bits derived from it (RefLib.symbol_chain_stats)",
            "rows": rows}
    (HERE / "ref_symbol_chain_curve.json").write_text(json.dumps(meta, indent=1))


MC_SNRS = list(range(0, 17)) + [18, 20, 22, 24, 26, 28, 30]
MC_DEEP_SNRS = (11, 12, 13, 14, 15)     # the BER waterfall, where the curve is set by rare sync failures
MC_DEEP_SCALE = {13: 4, 14: 4, 15: 4}   # x --mc-deep-trials where the 1e-3.5 .. 1e-5 crossings are pinned
MC_DEEP_JOB = 25_000                    # trials per deep job (seeded by job index: independent of --procs)


def _mc_worker(args):
    snr, n, seed = args
    R = RefLib()
    t, acc = R.mc_trials(snr, n, seed)
    return snr, n, t, acc.tolist()


def mc_jobs(trials: int, procs: int, deep_trials: int, deep_snrs=MC_DEEP_SNRS):
    """(snr, trials, seed) jobs.  Shallow points: `procs` jobs of trials // procs each, seeded
    1000003 (p + 1) + snr (the round-2 fixture's seeds: 48000 = 8 x 6000 reproduces its rows).  Deep
    points: deep_trials (x MC_DEEP_SCALE) in jobs of MC_DEEP_JOB, seeded 2000003 (j + 1) + snr."""
    jobs = []
    for s in MC_SNRS:
        if deep_trials and s in deep_snrs:
            n_jobs = MC_DEEP_SCALE.get(s, 1) * deep_trials // MC_DEEP_JOB
            jobs += [(float(s), MC_DEEP_JOB, 2000003 * (j + 1) + s) for j in range(n_jobs)]
        else:
            per = max(1, trials // procs)
            jobs += [(float(s), per, 1000003 * (p + 1) + s) for p in range(procs)]
    return jobs


def gen_mc(trials: int, procs: int, deep_trials: int):
    jobs = mc_jobs(trials, procs, deep_trials)
    jobs.sort(key=lambda j: -j[1])                      # long jobs first
    with mp.Pool(procs) as pool:
        res = list(pool.imap_unordered(_mc_worker, jobs, chunksize=1))
    curve = {}
    keys = ("sum_evm_db", "sum_evm_agc_db", "sum_ber", "sum_ber2", "trials_ber_pos", "trials_ber_ge_quarter",
            "sum_evm_db2", "trials_evm_agc_finite")
    for snr, n, t, acc in res:
        c = curve.setdefault(snr, {"trials": 0, "sec": 0.0, **{k: 0.0 for k in keys}})
        c["trials"] += n
        c["sec"] += t
        for k, v in zip(keys, acc):
            c[k] += v
    rows = []
    for snr in sorted(curve):
        c = curve[snr]
        n = c["trials"]
        var_ber = max(c["sum_ber2"] / n - (c["sum_ber"] / n) ** 2, 0.0)
        rows.append({"snr_db": snr, "trials": n, "ber": c["sum_ber"] / n,
                     "ber_trial_var": var_ber,                       # per-trial BER variance (frame-clustered)
                     "trials_ber_pos": int(c["trials_ber_pos"]),      # trials with any bit error
                     "trials_ber_ge_quarter": int(c["trials_ber_ge_quarter"]),   # failed frames (sync loss)
                     "mean_evm_db": c["sum_evm_db"] / n,
                     "evm_db_trial_var": max(c["sum_evm_db2"] / n - (c["sum_evm_db"] / n) ** 2, 0.0),
                     "mean_evm_agc_db": c["sum_evm_agc_db"] / n,
                     "trials_evm_agc_finite": int(c["trials_evm_agc_finite"]),
                     "sec_per_trial": c["sec"] / n})
    meta = {"generator": f"tests/golden/gen_golden.py --only mc --mc-trials {trials} --procs {procs} "
                         f"--mc-deep-trials {deep_trials}",
            "source": "reference OFDM.c (gcc -O2) TOA+Receiver loop (ref_harness.c ref_mc_trials)",
            "rand": "64-bit LCG hook (oracle/ref_harness.c)",
            "seeds": "shallow points: 1000003 (p + 1) + snr per process p; deep points "
                     f"{list(MC_DEEP_SNRS)} (x {MC_DEEP_SCALE} trials): {MC_DEEP_JOB}-trial jobs seeded "
                     "2000003 (j + 1) + snr",
            "rows": rows}
    (HERE / "ref_mc_curve.json").write_text(json.dumps(meta, indent=1))


def main():
    ap = argparse.ArgumentParser()
    # the defaults reproduce the committed ref_mc_curve.json (48000 trials/point, 1e6 at 11, 12 dB, 4e6 at 13, 14, 15)
    ap.add_argument("--mc-trials", type=int, default=48000)
    ap.add_argument("--mc-deep-trials", type=int, default=1_000_000)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--skip-mc", action="store_true")
    ap.add_argument("--only", choices=["genie", "mc", "chain"], help="regenerate one fixture only")
    a = ap.parse_args()
    build_ref()
    R = RefLib()
    if a.only == "genie":
        gen_genie(R)
        return
    if a.only == "mc":
        gen_mc(a.mc_trials, a.procs, a.mc_deep_trials)
        return
    if a.only == "chain":
        gen_chain(a.procs)
        return
    gen_fft(R); gen_tx(R); gen_rx(R); gen_kat(); gen_genie(R); gen_chain(a.procs)
    if not a.skip_mc:
        gen_mc(a.mc_trials, a.procs, a.mc_deep_trials)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
