#!/usr/bin/env python3
"""Benchmark: OFDM symbols/sec over the BER-vs-SNR sweep on MI355X (BASELINE.json metric).

One step = one full sweep of the hot path over one batch: the Tx pass (K2, data symbols written to
HBM once per chunk, OFDM.c:1191) and the per-SNR over-the-air + receive pass (K3, 16 SNR points
0..30 dB, OFDM.c:1202-1211) for every frame, then ONE all-reduce of the int64 counters.  Inputs (the
Tx batch) live in HBM for the whole step.  `value` = data OFDM symbols received and scored per
second over the whole job (symbols x SNR points / wall).

Workloads (BASELINE.json configs; --workload):
  c3 (default, configs[2]) real AWGN, LTF least squares + ZF + slicer + EVM, 1e7 symbols/point per
     GPU (weak scaling: the largest single-GPU config; the driver's 1/2/4/8-GPU curve runs this)
  c2 (configs[1])          ideal CSI, 1e6 symbols/point, 1 GPU
  c4 (configs[3])          c3's chain, 1e8 symbols/point in TOTAL, split over the ranks (strong)
  c5 (configs[4])          1e9 symbol-SNR evaluations in TOTAL (6.25e7 symbols/point x 16 points; not 1e9
                           symbols per point), split over the ranks (strong): 4-tap Rayleigh + ZF (LS), real
                           AWGN (every config uses the reference's real-only noise)
  frame                    the reference's own trial (sync, CFO, LS): the like-for-like line next
                           to the reference's trial loop on the host
  fft64                    K1 alone (ofdm_fft64, OFDM.c fft()/ifft() :282-339): 2^24 64-point transforms per launch,
                           a step = one fft + one ifft over the HBM-resident batch; HBM roofline at 1,024 B per
                           transform (512 B read + 512 B written); units are transforms (one OFDM symbol each)

Launched as `python bench.py --gpus N --steps K --warmup W`.  For N > 1 outside torchrun, bench.py starts
`torch.distributed.run --nproc-per-node N` on itself as a child process (launch_ranks; it never execs) and
relays rank 0's line; under torchrun every rank checks WORLD_SIZE == --gpus.  One rank per GPU, RCCL all-reduce
of the counters; OFDM_DIST_BACKEND=gloo reduces host copies instead (several ranks sharing one GPU: the tests'
world-2 run on a 1-GPU box).  Rank 0 prints ONE JSON line.
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
# wave64 VALU issue peak: 256 CUs x 4 SIMDs x 1 wave-instruction per 2 cycles at 2.4 GHz
# (MI355X_MICROARCH.md "Wave scheduling"; tools/ubench_valu.hip)
VALU_PEAK_GHZ = 2.4
VALU_PEAK_PER_S = 256 * 4 * 0.5 * VALU_PEAK_GHZ * 1e9
# capture samples read per trial (complex f32, from the L2-resident waveform): 3008 for the reference message,
# int(0.307 x 19400) = 5955 for frame8's 8-symbol waveform (OFDM.c:945)
FRAME_CAPTURE_SAMPLES = {"frame": 3008, "frame8": 5955}
SNR_GRID = np.arange(0.0, 31.0, 2.0)
MAX_CHUNK_FRAMES = 1 << 23         # largest device-resident Tx batch (16.8M symbols, 10.7 GB of HBM)
PIPE_CHUNKS = 4                    # Tx / receiver pipeline depth of a step (symbol workloads)
MIN_PIPE_FRAMES = 1 << 18          # smaller chunks are not split further

_LS_AWGN = dict(est="ls", noise="real", channel="awgn", conv="c", payload="random")
WORKLOADS = {
    # name: description, cfg kwargs, data symbols per SNR point, scaling ("weak": per GPU, "strong": total)
    "c3": ("BASELINE configs[2]: AWGN sweep 0-30 dB step 2 + LTF LS channel est + slicer/EVM, 1e7 symbols/point "
           "per GPU", _LS_AWGN, 10_000_000, "weak"),
    "c2": ("BASELINE configs[1]: AWGN BER sweep 0-30 dB step 2, ideal channel, 1e6 symbols/point",
           dict(est="ideal", noise="real", channel="awgn", conv="c", payload="random"), 1_000_000, "weak"),
    "c4": ("BASELINE configs[3]: c3's chain, 1e8 symbols/point in total, counter-range shards over the ranks, "
           "RCCL all-reduce of the int64 counters", _LS_AWGN, 100_000_000, "strong"),
    "c5": ("1e9 symbol-SNR evaluations in total (6.25e7 symbols/point x 16 SNR points, split over the ranks) -- "
           "BASELINE configs[4]: 4-tap Rayleigh + per-subcarrier ZF (LTF LS), real AWGN, full BER/EVM sweep",
           dict(est="ls", noise="real", channel="rayleigh4", conv="c", payload="random"),
           62_500_000, "strong"),
    "frame": ("frame mode: OFDM.c Transmission_Over_Air + Receiver trials (sync, CFO, LS), reference message; the "
              "capture's tail is generated only when the first detection round does not decide Packet_Selection "
              "(results bit-identical to full evaluation, OFDM_FRAME_NO_LAZY)",
              dict(payload="message", noise="real", conv="c"), 1_000_000, "weak"),
    "frame8": ("frame mode with a 96-character message (8 data symbols per frame, 5955-sample captures: the long-"
               "message path); units are data symbols x SNR points",
               dict(payload="message", noise="real", conv="c"), 1_000_000, "weak"),
    "fft64": ("K1: batched 64-point fft() + ifft() (C convention) of HBM-resident symbols, 2^24 transforms per "
              "launch", {}, 1 << 24, "weak"),
}
COLLECTIVE = {"nccl": "RCCL", "gloo": "gloo (host copy)"}
FFT_BYTES_PER_TRANSFORM = 1024     # 64 complex f32 read + 64 written
STEP_DEFAULTS = {"c2": (50, 10)}   # (steps, warmup) when not given
# data symbols per frame (trial) of each workload; frame8 sets its message before the sweep
FRAME_DATA = {"frame8": 8}
FRAME8_MESSAGE = (b"The quick brown fox jumps over the lazy dog; 802.11a OFDM-QPSK frames on MI355X, eight symbols.. ")[:96]


def load_pmc(workload: str) -> dict:
    """Per-launch rocprofv3 --pmc figures for this workload (profiles/pmc_summary.json, written by
    tools/pmc_summary.py from tools/gpu_profile.sh runs), or {}."""
    p = ROOT / "profiles" / "pmc_summary.json"
    try:
        # c4 launches c3's receiver on c3's configuration (only the chunking differs): c3's counters apply
        return json.loads(p.read_text()).get({"c4": "c3"}.get(workload, workload), {})
    except Exception:
        return {}


def issue_cap(pmc: dict, frac: float) -> dict:
    """The instruction-mix cap of the kernel's loop (tools/isa_mix.py --record: class-priced issue cycles of
    its gfx950 assembly) and this run's fraction of it, when recorded."""
    m = pmc.get("issue_model")
    if not m:
        return {}
    if m.get("method") == "dynamic":     # tools/mix_cap.py: the measured class mix, ambiguous classes bounded
        lo, hi = m["cap_frac_range"]
        return {"issue_model_cap_frac": lo, "issue_model_cap_frac_range": [lo, hi],
                "frac_of_issue_model_cap": frac / lo, "frac_of_issue_model_cap_range": [frac / hi, frac / lo],
                "issue_model_note": "cap = 2 x VALU / SIMD cycles of the dynamic class mix (PMC class counters) at "
                                    "%s waves/SIMD, unclassified instructions priced slow (cap) or fast (upper end)"
                                    % m["waves_per_simd"]}
    if m.get("method") == "dynamic_split":   # tools/mix_cap.py --split-from: a point estimate inside that range
        lo, hi = m["cap_frac_range"]
        return {"issue_model_cap_frac": m["cap_frac"], "issue_model_cap_frac_range": [lo, hi],
                "frac_of_issue_model_cap": frac / m["cap_frac"], "frac_of_issue_model_cap_range": [frac / hi, frac / lo],
                "issue_model_note": "cap = 2 x VALU / SIMD cycles of the dynamic class mix (PMC class counters) at "
                                    "%s waves/SIMD, the unclassified instructions split fast / slow / cndmask as in "
                                    "the classified model of frame's sync kernel (%s); range: all slow .. all fast"
                                    % (m["waves_per_simd"], m["split_source"])}
    if m.get("method") == "classified":  # tools/frame_mix.py / frame8_mix.py: every VALU instruction classified
        return {"issue_model_cap_frac": m["cap_frac"], "frac_of_issue_model_cap": frac / m["cap_frac"],
                "issue_model_note": "cap = 2 x VALU / class-priced SIMD cycles at %s waves/SIMD of both kernels' "
                                    "assembly, blocks weighted per item (undecided fraction %.3f fitted to the "
                                    "measured %s)" % (m["waves_per_simd"], m["undecided_fraction"],
                                                      m.get("fit", "SQ_INSTS_VALU"))}
    return {"issue_model_cap_frac": m["cap_frac"], "frac_of_issue_model_cap": frac / m["cap_frac"],
            "issue_model_note": "cap = 2 x loop VALU / class-priced SIMD cycles at %s waves/SIMD (modelled)"
                                % m["waves_per_simd"]}


def certify_pmc(pmc: dict, kernel: str, lib_id: str | None) -> tuple[dict, str | None]:
    """The PMC record only if it measured THIS build of THIS kernel: same kernel set and the same build id
    (codeobj: hash of the kernels' gfx950 code + descriptors) as the library this run loaded.  Otherwise
    ({}, reason): a stale instruction count never reaches the roofline."""
    if not pmc:
        return {}, "no PMC record for this workload"
    if "+".join(pmc.get("kernels", [pmc.get("kernel")])) != kernel:
        return {}, f"PMC record is of {pmc.get('kernels')}, this run launches {kernel}"
    if lib_id is None:
        return {}, "kernel not found in the loaded library's gfx950 code objects"
    if pmc.get("build_id") != lib_id:
        return {}, f"PMC record build id {pmc.get('build_id')} != loaded library's {lib_id} (stale record)"
    return pmc, None


def make_roofline(pmc: dict, lib_id: str | None, kernel: str, workload: str, units_per_launch: float,
                  rx_avg_s: float, rx_n: int, fused_tx: bool) -> tuple[dict, float | None]:
    """The VALU-issue roofline of the run's receiver: achieved = measured VALU wave-instructions per unit
    (SQ_INSTS_VALU / units, rocprofv3 --pmc, profiles/pmc_summary.json) x this run's units per launch / this
    run's mean launch time (HIP events on the launch stream).  frac is null unless the PMC record is
    certified for the loaded build (certify_pmc).  Returns (roofline, measured HBM bytes per launch)."""
    pmc, why = certify_pmc(pmc, kernel, lib_id)
    ipu = pmc.get("valu_instr_per_unit")
    tpu = pmc.get("hbm_bytes_per_unit")
    traffic = tpu * units_per_launch if tpu else None
    base = {"bound": "valu", "peak": VALU_PEAK_PER_S, "unit": "wave-instr/s", "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (PMC)", "kernel": kernel, "avg_launch_ms": rx_avg_s * 1e3,
            "launches": rx_n, "units_per_launch": units_per_launch, "lib_build_id": lib_id,
            "pmc_build_id": pmc.get("build_id")}
    if not ipu:
        return {**base, "achieved": None, "frac": None, "frac_null_reason": why or "no VALU count"}, traffic
    achieved = units_per_launch * ipu / rx_avg_s
    frac = achieved / VALU_PEAK_PER_S
    model = pmc.get("issue_model")
    cap = issue_cap(pmc, frac) if model and model.get("build_id") == lib_id else {}
    # the nominal peak assumes 2.4 GHz; the certified PMC run of the same command measured the SQ clock
    # (GRBM_GUI_ACTIVE per XCD over the receiver dispatches): the same fractions at that clock separate the
    # clock from the issue efficiency (this run's own clock is not measured)
    clk = pmc.get("clock_ghz")
    if clk and clk == clk:
        scale = VALU_PEAK_GHZ / clk
        cap = {**cap, "profiled_clock_ghz": clk, "frac_at_profiled_clock": frac * scale,
               **({"frac_of_issue_model_cap_at_profiled_clock": cap["frac_of_issue_model_cap"] * scale}
                  if "frac_of_issue_model_cap" in cap else {})}
    return {**base, "achieved": achieved, "frac": frac, "instr_per_unit": ipu,
            "pmc_source": "profiles/pmc_summary.json[%s]" % {"c4": "c3"}.get(workload, workload),
            **({"fused_tx": "the receivers build the step's Tx batches: chunk 0's its own (ofdm_txrx_frames), "
                            "chunk k's the batch of chunk k+1 (ofdm_set_next_tx); their VALU and HBM counts include "
                            "it"} if fused_tx else {}),
            **cap}, traffic


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _cgroup_cpu_quota() -> tuple[float | None, str]:
    """CPUs granted by the cgroup CPU quota (v2 cpu.max, v1 cfs_quota_us / cfs_period_us), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            return int(q) / int(per), f"cgroup v2 cpu.max {q}/{per}"
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        if q > 0:
            return q / per, f"cgroup v1 cfs quota {q}/{per}"
    except (OSError, ValueError):
        pass
    return None, "no cgroup CPU quota"


def host_cpu_share() -> dict:
    """The host CPUs this job may use, derived rather than assumed: the scheduler affinity mask, capped by
    the cgroup CPU quota when one is set.  Under torchrun the share belongs to the whole job (one node),
    and local rank 0 times the reference on all of it while the other ranks wait at the rendezvous."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    quota, src = _cgroup_cpu_quota()
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return {"cores": cores, "affinity": aff, "quota": quota, "source": src, "visible": os.cpu_count() or aff}


def _trial_worker(args):
    """The reference's own trial loop: (symbols, seconds, mean BER)."""
    snr, n, seed = args
    from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
    t, acc = RefLib().time_trials(snr, n, seed)
    return 2 * n, t, float(acc[2]) / n


def _chain_worker(args):
    """The symbol chain built from the reference's stage functions: (symbol-SNR units, seconds, BER)."""
    n, seed, rayleigh, ideal = args
    from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
    t, acc = RefLib().time_symbol_chain(SNR_GRID, n, rayleigh=rayleigh, seed=seed, ideal=ideal)
    return 2 * n * len(SNR_GRID), t, float(acc[0] / max(acc[1], 1))


def _barrier_proc(worker, args, barrier, queue):
    """Spawned host process: load the reference library, wait until every process is ready, then
    run the timed loop (so process start-up is outside every timed region)."""
    from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
    RefLib()
    barrier.wait()
    w0 = time.perf_counter()
    r = worker(args)
    queue.put((r, w0, time.perf_counter()))


def _parallel(worker, jobs) -> tuple[float, float, list]:
    """Run the jobs in len(jobs) spawned processes started together: (units, wall seconds, results)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    barrier, queue = ctx.Barrier(len(jobs)), ctx.Queue()
    procs = [ctx.Process(target=_barrier_proc, args=(worker, j, barrier, queue)) for j in jobs]
    for pr in procs:
        pr.start()
    out = [queue.get(timeout=600) for _ in procs]
    for pr in procs:
        pr.join()
    wall = max(o[2] for o in out) - min(o[1] for o in out)
    return sum(o[0][0] for o in out), wall, [o[0] for o in out]


def cpu_baseline(workload: str, seconds: float = 12.0, share: dict | None = None) -> dict | None:
    """The reference itself (oracle/_ref/libofdm_ref.so, the unmodified OFDM.c built with gcc -O2,
    kind "reference") timed on this host, on the workload's own chain:
      frame            its trial loop (Transmission_Over_Air + Receiver, OFDM.c:1206-1217) at 10 dB;
      c3/c4/c5         the genie symbol chain of the GPU sweep composed from its stage functions
                       (QPSK_Modulator, ifft, gaussian_noise, Channel_Estimation, fft, AGC_Receiver,
                       QPSK_Demodulator; ref_harness.c ref_time_symbol_chain) over the same 16 SNR
                       points, the Tx built once per frame as the GPU re-uses its Tx batch (c5 adds
                       a restated 4-tap channel ahead of the noise: the reference has none, D9);
      c2               the same chain with the known channel (ideal CSI): no per-SNR Channel_Estimation,
                       as the GPU's ideal-CSI receiver has none.
    The reference is single-threaded with global state, so the multi-core figure runs one process
    per CPU of the job's host share (host_cpu_share: affinity capped by the cgroup quota); the
    one-thread figure is reported beside it.  Runs before the GPU is initialised."""
    try:
        from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
        ref = RefLib()
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "OFDM symbols/s", "cores": 0, "kind": "reference",
                "sample": f"unavailable: {e}"}
    if workload == "fft64":
        return cpu_baseline_fft(ref, seconds, share)
    frame = workload.startswith("frame")     # frame8: the reference has only its own 2-symbol message
    rayleigh = workload == "c5"
    ideal = workload == "c2"
    if frame:
        t, _ = ref.time_trials(10.0, 50, 1)
        per = max(t / 50, 1e-6)
        one = lambda n, s: _trial_worker((10.0, n, s))  # noqa: E731
        job = lambda n, s: (10.0, n, s)                 # noqa: E731
        worker = _trial_worker
        what = ("reference trials (Transmission_Over_Air + Receiver of src/OFDM.c, frame mode, 2 data symbols "
                "each) at SNR 10 dB")
    else:
        t, _ = ref.time_symbol_chain(SNR_GRID, 20, rayleigh=rayleigh, seed=1, ideal=ideal)
        per = max(t / 20, 1e-6)
        one = lambda n, s: _chain_worker((n, s, rayleigh, ideal))  # noqa: E731
        job = lambda n, s: (n, s, rayleigh, ideal)                 # noqa: E731
        worker = _chain_worker
        est = "known channel (ideal CSI)" if ideal else "LTF LS"
        what = (f"frames of the genie symbol chain composed from src/OFDM.c's stage functions "
                f"({'4-tap Rayleigh, ' if rayleigh else ''}{est}, 2 data symbols each) x "
                f"{len(SNR_GRID)} SNR points")
    cpu = cpu_model()
    share = share or host_cpu_share()
    P = share["cores"]
    n1 = max(20, int(seconds / 3 / per))
    u1, t1, m1 = one(n1, 7)
    single = {"value": u1 / t1, "unit": "OFDM symbols/s", "cores": 1, "kind": "reference",
              "sample": f"{n1} {what} on 1 thread in {t1:.1f} s; mean BER {m1:.3g}"}
    n = max(20, int(seconds * 2 / 3 / per))
    units, wall, res = _parallel(worker, [job(n, 1000 + k) for k in range(P)])
    return {"value": units / wall, "unit": "OFDM symbols/s", "cores": P, "kind": "reference",
            "sample": f"{P} x {n} {what} in {wall:.1f} s wall on {P} host processes started together "
                      f"(start-up untimed); mean BER {sum(r[2] for r in res) / P:.3g}",
            "cpu_model": cpu, "cpus_visible": share["visible"],
            "cores_source": f"{P} = min(sched_getaffinity {share['affinity']}, {share['source']})",
            "cores_note": ("measured on the job's whole host share; CPUs outside it belong to other jobs "
                           "and are not used (no extrapolation)"),
            "single_core": single}


def _fft_worker(args):
    """The reference's fft() then ifft() on n vectors: (transforms, seconds, checksum)."""
    n, seed = args
    from oracle import RefLib  # noqa: PLC0415  (bench.py's cpu_baseline leg only)
    r = RefLib()
    t1, c1 = r.time_fft(n, False, seed=seed)
    t2, c2 = r.time_fft(n, True, seed=seed)
    return 2 * n, t1 + t2, c1 + c2


def cpu_baseline_fft(ref, seconds: float, share: dict | None) -> dict:
    """fft64: the reference's own fft() / ifft() (OFDM.c:282-339, gcc -O2) on the host, one process per CPU of the
    job's share and on one thread, the same alternation of fft and ifft as the GPU step."""
    t, _ = ref.time_fft(20000, False)
    per = max(t / 20000, 1e-9)
    share = share or host_cpu_share()
    P = share["cores"]
    n1 = max(1000, int(seconds / 6 / per))
    u1, t1, _ = _fft_worker((n1, 7))
    single = {"value": u1 / t1, "unit": "OFDM symbols/s", "cores": 1, "kind": "reference",
              "sample": f"{n1} fft() + {n1} ifft() calls of src/OFDM.c on 64 samples, 1 thread, {t1:.1f} s"}
    n = max(1000, int(seconds / 3 / per))
    units, wall, _ = _parallel(_fft_worker, [(n, 1000 + k) for k in range(P)])
    return {"value": units / wall, "unit": "OFDM symbols/s", "cores": P, "kind": "reference",
            "sample": f"{P} x ({n} fft() + {n} ifft()) of src/OFDM.c on 64 samples in {wall:.1f} s wall on {P} host "
                      "processes started together (start-up untimed)",
            "cpu_model": cpu_model(), "cpus_visible": share["visible"],
            "cores_source": f"{P} = min(sched_getaffinity {share['affinity']}, {share['source']})",
            "single_core": single}


def plan_chunks(first: int, frames: int, n_chunks: int = 0) -> list[tuple[int, int]]:
    """Equal chunks (no small tail launch) of at most MAX_CHUNK_FRAMES frames, and at least PIPE_CHUNKS of
    them (each >= MIN_PIPE_FRAMES) so that the Tx of chunk k+1 can be built under the receiver of chunk k
    (n_chunks > 0: that many, at least as many as MAX_CHUNK_FRAMES needs)."""
    auto = PIPE_CHUNKS if frames >= PIPE_CHUNKS * MIN_PIPE_FRAMES else 1
    n_chunks = max(n_chunks or auto, -(-frames // MAX_CHUNK_FRAMES))
    cut = [first + frames * k // n_chunks for k in range(n_chunks + 1)]
    return [(cut[k], cut[k + 1] - cut[k]) for k in range(n_chunks) if cut[k + 1] > cut[k]]


class PipelinedSymbolStep:
    """One symbol-mode step: Tx + receiver of every chunk into two alternating Tx batches.  `fused` (the packed
    real-noise receivers): the receivers build every batch, one stream -- chunk 0's receiver its own batch
    (ofdm_txrx_frames: each group's symbols built in its prologue, then read back) and the receiver of chunk k
    chunk k+1's batch (ofdm_set_next_tx, on the waves that idle while the clean spectra are transformed).
    Otherwise the Tx of chunk k+1 runs on a second stream while the receiver of chunk k runs
    (tools/overlap_ab.py: c3 +1.5-2.7 %, counters bit-identical); events order each batch's reuse after the
    receiver that read it, and a step's Tx stream after every receiver of the previous step."""

    def __init__(self, torch, eng, cfg, chunks, counters, dev: int, fused: bool = False):
        self.torch, self.eng, self.cfg, self.chunks, self.counters = torch, eng, cfg, chunks, counters
        self.bufs = [eng.tx_buffers(max(n for _, n in chunks)) for _ in range(2 if len(chunks) > 1 else 1)]
        self.s_rx = torch.cuda.current_stream(dev)
        self.s_tx = torch.cuda.Stream(dev)
        self.fused = fused

    def __call__(self):
        torch, eng, cfg, chunks, bufs = self.torch, self.eng, self.cfg, self.chunks, self.bufs
        s_rx, s_tx = self.s_rx, self.s_tx
        self.counters.zero_()
        if self.fused:
            # one stream: the batch receiver k overwrites (chunk k+1's) was last read by receiver k-1
            eng.set_stream(s_rx.cuda_stream)
            for k, (a, n) in enumerate(chunks):
                if k + 1 < len(chunks):
                    eng.set_next_tx(cfg, chunks[k + 1][0], chunks[k + 1][1], *bufs[(k + 1) % 2])
                if k == 0:
                    eng.txrx_frames(cfg, a, n, SNR_GRID, *bufs[0], self.counters)
                else:
                    eng.rx_frames(cfg, *bufs[k % 2], a, n, SNR_GRID, self.counters)
            return
        tx_done = [torch.cuda.Event() for _ in chunks]
        rx_done = [torch.cuda.Event() for _ in chunks]
        start = torch.cuda.Event()
        start.record(s_rx)
        s_tx.wait_event(start)                           # after every receiver of the previous step
        eng.set_stream(s_rx.cuda_stream)
        eng.tx_frames(cfg, chunks[0][0], chunks[0][1], *bufs[0])
        for k, (a, n) in enumerate(chunks):
            if k + 1 < len(chunks):                      # Tx of the next chunk into the other buffer
                if k >= 1:
                    s_tx.wait_event(rx_done[k - 1])      # ... once the receiver of chunk k-1 has read it
                eng.set_stream(s_tx.cuda_stream)
                eng.tx_frames(cfg, chunks[k + 1][0], chunks[k + 1][1], *bufs[(k + 1) % 2])
                tx_done[k + 1].record(s_tx)
                eng.set_stream(s_rx.cuda_stream)
            if k >= 1:
                s_rx.wait_event(tx_done[k])
            eng.rx_frames(cfg, *bufs[k % 2], a, n, SNR_GRID, self.counters)
            rx_done[k].record(s_rx)


def run_fft64(args, cpu, torch, dist, pkg, abi, codeobj, rank, world, dev, distributed, backend):
    """--workload fft64: K1 (ofdm_fft64) alone on an HBM-resident batch of 2^24 symbols per GPU (weak scaling).  A
    step is fft() of the batch into a second buffer and ifft() back (C convention, OFDM.c:314-339): two launches,
    2^25 transforms.  The roofline is HBM: 1,024 algorithmic bytes per transform over the launches' HIP-event time
    against 8 TB/s; `traffic` is the PMC-measured FETCH_SIZE x 2 + WRITE_SIZE per launch when a record of this build
    exists (profiles/pmc_summary.json["fft64"])."""
    desc, _, n, scaling = WORKLOADS["fft64"]
    if args.symbols:
        n = args.symbols
    eng = pkg.Engine(dev)
    g = torch.Generator(device=f"cuda:{dev}").manual_seed(0x80211A + rank)
    x = torch.randn((n, 64), dtype=torch.complex64, device=f"cuda:{dev}", generator=g)
    y = torch.empty_like(x)
    done = torch.zeros(1, dtype=torch.int64, device=f"cuda:{dev}")

    def step():
        eng.fft64_into(x, y, inverse=False)
        eng.fft64_into(y, x, inverse=True)
        if distributed:
            host_allreduce(dist, done, dist.ReduceOp.SUM)    # the job's one collective (a completion count)

    x0 = x[:4].clone()
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
    ms, launches = eng.timing_query(abi.K_FFT)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        elapsed = host_allreduce(dist, t, dist.ReduceOp.MAX).item()
    # ifft(fft(x)) in the reference's C convention is x circularly shifted by 32 samples (fftshift of the IDFT,
    # SURVEY D5): after an odd number of steps the first vectors are x0 rolled by 32, after an even number x0 (a
    # cheap check that the launches did the work)
    want = x0.roll(32, dims=1) if (args.warmup + args.steps) % 2 else x0
    rt_err = float((x[:4] - want).abs().max() / x0.abs().max())
    units_per_launch = float(n)
    avg_s = ms / max(launches, 1) / 1e3
    achieved = units_per_launch * FFT_BYTES_PER_TRANSFORM / avg_s / 1e9
    pmc = load_pmc("fft64")
    lib_id = codeobj.workload_build_id(abi.library_file(), "fft64")
    cert, why = certify_pmc(pmc, "fft64_lds_kernel", lib_id)
    tpu = cert.get("hbm_bytes_per_unit")
    value = 2.0 * n * world * args.steps / elapsed
    if rank == 0:
        line = {
            "metric": "OFDM symbols/sec (whole node) over BER-vs-SNR sweep; achieved HBM GB/s vs peak",
            "value": value, "unit": "OFDM symbols/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (torch.randn complex64, seed 0x80211A + rank)",
            "config": {"workload": "fft64", "description": desc, "transforms_per_launch_per_gpu": n,
                       "launches_per_step": 2, "conv": "c",
                       "parallelism": (f"dp{world} (each rank its own batch, weak scaling; 1 {COLLECTIVE[backend]} "
                                       "all-reduce of a completion count per step)" if distributed
                                       else "1 process, no collective (not launched under torchrun)"),
                       "backend": backend if distributed else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": tpu * units_per_launch if tpu else None,
                         "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE)",
                         **({"traffic_null_reason": why} if not tpu else {}),
                         "algorithmic_bytes_per_unit": FFT_BYTES_PER_TRANSFORM, "kernel": "fft64_lds_kernel",
                         "avg_launch_ms": avg_s * 1e3, "launches": launches, "units_per_launch": units_per_launch,
                         "lib_build_id": lib_id, "pmc_build_id": pmc.get("build_id")},
            "results": {"fft_ifft_roundtrip_max_rel_err": rt_err},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    eng.close()
    if distributed:
        dist.destroy_process_group()


def wants_cpu_baseline(args) -> bool:
    """Rank 0 of the job times the reference (any WORLD_SIZE); the others do not.  A self-launching parent
    (launch_ranks) never does: its rank 0 child does."""
    return int(os.environ.get("RANK", "0")) == 0 and not args.no_cpu_baseline


def _free_port() -> int:
    import socket  # noqa: PLC0415
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_command(n: int, argv: list[str], port: int) -> list[str]:
    """The torchrun command line of `bench.py --gpus n` started outside torchrun: one rank per GPU of this node,
    rendezvous on 127.0.0.1, the same bench arguments (each rank then sees WORLD_SIZE == --gpus)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), *argv]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`--gpus n > 1` outside torchrun: start the n ranks under torch.distributed.run as a CHILD process (this
    process never touches the GPU and never execs), pass its output through and relay rank 0's JSON line as the
    one line on stdout.  Returns the child's exit status (non-zero also when no JSON line came back)."""
    import subprocess  # noqa: PLC0415
    cmd = child_command(n, argv, _free_port())
    print("bench.py: launching %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=str(ROOT))
    lines = []
    for ln in proc.stdout:                 # streamed: progress reaches the log while the ranks run
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            lines.append(s)
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: the {n}-rank child exited with {rc}", file=sys.stderr)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def check_world(args) -> None:
    """Under torchrun every rank must see WORLD_SIZE == --gpus: a line's n_gpus is the world size, so a mismatch
    would report a different job than the one asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")


def host_allreduce(dist, t, op):
    """all_reduce of a device tensor through a host copy (gloo: several ranks sharing one GPU, or CPU tests);
    RCCL reduces it in HBM"""
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=op)
        return t
    h = t.cpu()
    dist.all_reduce(h, op=op)
    t.copy_(h)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 5; c2 50)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warm-up steps (default: 2; c2 10)")
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--symbols", type=int, default=0,
                    help="override data symbols per SNR point (per GPU for weak workloads, total for strong)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--chunks", type=int, default=0, help="Tx/receiver chunks per step (0: plan_chunks)")
    ap.add_argument("--pipeline", choices=("auto", "fused", "streams"), default="auto",
                    help="next chunk's Tx: fused into the LS receiver (auto for real-noise LS) or a second stream")
    args = ap.parse_args()
    # c2's step is one ~1 ms launch: 5 steps would time mostly the clock ramp (1.94 GHz in the first launches, 2.36 in
    # the last), so its defaults are longer; every other workload's step is >= 6 ms
    dflt = STEP_DEFAULTS.get(args.workload, (5, 2))
    args.steps = dflt[0] if args.steps is None else args.steps
    args.warmup = dflt[1] if args.warmup is None else args.warmup
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "RANK" not in os.environ and args.gpus > 1:
        # one rank per GPU: this process only launches them (nothing here touches the GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    check_world(args)

    # host-side reference timing first, before anything touches the GPU (worker processes are spawned).
    # Under torchrun rank 0 (local rank 0 of the one node) times it before forming the process group; the
    # other ranks wait at the rendezvous, so every N-GPU line carries the CPU figure of the same run
    cpu = cpu_baseline(args.workload, args.cpu_seconds) if wants_cpu_baseline(args) else None

    import torch
    import torch.distributed as dist
    pkg = ofdm_pkg.load()
    from ofdm_amd import abi, codeobj, dist as odist

    rank, world, local = odist.env_rank_world()
    # under torch.distributed.run (RANK set) the group is formed even for one rank, and the counters' all-reduce
    # runs through it: RCCL (one rank per GPU), or gloo with OFDM_DIST_BACKEND=gloo (ranks may share a GPU)
    distributed = "RANK" in os.environ
    backend = os.environ.get("OFDM_DIST_BACKEND", "nccl")
    dev = 0
    if distributed:
        dev = local if backend == "nccl" else local % max(torch.cuda.device_count(), 1)
        odist.init_from_env(backend, device=dev)
        torch.cuda.set_device(dev)

    if args.workload == "fft64":
        run_fft64(args, cpu, torch, dist, pkg, abi, codeobj, rank, world, dev, distributed, backend)
        return
    desc, kw, symbols, scaling = WORKLOADS[args.workload]
    if args.symbols:
        symbols = args.symbols
    dpf = FRAME_DATA.get(args.workload, 2)         # D data symbols per frame (2: OFDM.c:439)
    total_frames = symbols // dpf
    if scaling == "weak":
        first, end = odist.weak_range(total_frames, rank)
    else:
        first, end = odist.shard_range(total_frames, rank, world)
    frames = end - first
    cfg = pkg.make_cfg(**kw)
    eng = pkg.Engine(dev)
    frame_mode = args.workload.startswith("frame")
    if args.workload == "frame8":
        # not inside an assert: under python -O the message would silently stay the 2-symbol reference one
        got = eng.set_message(FRAME8_MESSAGE)
        if got != dpf:
            raise SystemExit(f"frame8: set_message framed {got} data symbols, expected {dpf}")
    counters = eng.new_counters(len(SNR_GRID))
    chunks = plan_chunks(first, frames, args.chunks)
    # real-noise sweeps on the packed receivers (c2, c3, c4, c5): every Tx batch built inside the receivers
    packed = kw.get("noise") == "real" and (kw.get("channel") == "awgn" or kw.get("est") == "ls")
    fused = packed if args.pipeline == "auto" else args.pipeline == "fused"
    sym_step = (PipelinedSymbolStep(torch, eng, cfg, chunks, counters, dev, fused=fused)
                if not frame_mode and chunks else None)

    frame_host = [None]           # frame mode's host counters of the last step (ofdm_frame_sweep returns them)

    def step():
        if frame_mode:            # one trial = one frame of dpf data symbols; waveform cached on the device
            frame_host[0] = eng.frame_sweep(cfg, SNR_GRID, frames, first_trial=first)
            if distributed:       # the all-reduce below works on the device tensor; one rank needs no device copy
                counters.copy_(torch.from_numpy(frame_host[0]))
        elif sym_step is not None:
            sym_step()
        else:
            counters.zero_()      # a rank without frames (strong split of a tiny job)
        if distributed:
            host_allreduce(dist, counters, dist.ReduceOp.SUM)   # RCCL over xGMI (a copy at world 1)

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
        elapsed = host_allreduce(dist, t, dist.ReduceOp.MAX).item()

    if frame_mode and not distributed:
        counters.copy_(torch.from_numpy(frame_host[0]))
    c = counters.cpu().numpy()
    n_snr = len(SNR_GRID)
    job_frames = total_frames * (world if scaling == "weak" else 1)
    total_units = float(job_frames) * dpf * n_snr * args.steps        # symbol-SNR evaluations, all ranks
    value = total_units / elapsed
    rx_avg_s = rx_ms / max(rx_n, 1) / 1e3
    units_per_launch = frames * dpf * n_snr * args.steps / max(rx_n, 1)  # this rank's units per receiver launch
    bytes_per_unit = FRAME_CAPTURE_SAMPLES[args.workload] * 8 / dpf if frame_mode else BYTES_PER_SYMBOL_SNR
    res = pkg.SweepResult(SNR_GRID, c)
    pmc = load_pmc(args.workload)
    # the receiver kernel this workload launches (ofdm_symbol.hip launch_rx): real-noise AWGN sweeps and
    # real-noise LS Rayleigh sweeps run the packed receiver (ofdm_rxpack.hip), the others the {E, D0, D1}
    # LS / ideal receivers
    # frames of >= 5 data symbols (captures > 4,100 samples) run the long-capture sync kernel (ofdm_frame_long.hip)
    kernel = (("frame_sync_long_kernel+frame_sym_kernel" if args.workload == "frame8" else "frame_sync_kernel+frame_sym_kernel")
              if frame_mode
              else "rx_pack_kernel" if kw.get("noise") == "real" and (kw.get("channel") == "awgn" or kw.get("est") == "ls")
              else ("rx_ls_kernel" if kw.get("est") == "ls" else "rx_ideal_kernel"))
    lib_id = codeobj.workload_build_id(abi.library_file(), args.workload)
    roofline, traffic = make_roofline(pmc, lib_id, kernel, args.workload, units_per_launch, rx_avg_s, rx_n,
                                      fused and not frame_mode)
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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox4x32-10 bits and noise, seed 0x80211A)",
            "config": {"workload": args.workload, "description": desc,
                       "symbols_per_snr": symbols if scaling == "strong" else symbols * world,
                       "symbols_per_snr_per_gpu": dpf * frames, "snr_db": SNR_GRID.tolist(),
                       "frames_per_gpu": frames, "data_symbols_per_frame": dpf, "chunks_per_step": len(chunks),
                       "parallelism": (f"dp{world} (counter-range shards, {scaling} scaling; 1 {COLLECTIVE[backend]} "
                                       "all-reduce of int64 counters per step)" if distributed
                                       else "1 process, no collective (not launched under torchrun)"),
                       "backend": backend if distributed else None},
            # the binding roofline: VALU issue (make_roofline)
            "roofline": roofline,
            # HBM: the measured traffic (PMC) against the HBM peak is the HBM roofline fraction.  SURVEY
            # §8(d)'s streaming figure (652 B per unit, as if each symbol were re-read per SNR point) is NOT
            # traffic: the kernels stage a symbol once per launch for all SNR points.  Only its per-unit size is
            # kept, with no rate, so that no field of the line reads as a bandwidth above the HBM peak
            "hbm": {"measured_bytes_per_launch": traffic,
                    "measured_gbs": traffic / rx_avg_s / 1e9 if traffic else None,
                    "measured_frac": traffic / rx_avg_s / 1e9 / HBM_PEAK_GBS if traffic else None,
                    "peak_gbs": HBM_PEAK_GBS,
                    "survey_streaming_bytes_per_unit": {
                        "bytes_per_unit": bytes_per_unit, "is_traffic": False,
                        "note": "SURVEY 8(d) per-unit size if every unit were streamed from HBM; the fused "
                                "kernels read each symbol once per launch (see measured_bytes_per_launch)"}},
            "kernels_ms": {"rx_total": rx_ms, "rx_launches": rx_n, "tx_total": tx_ms, "tx_launches": tx_n},
            "results": {"ber": res.ber.tolist(), "evm_pre_db": res.evm_pre_db.tolist(),
                        "frames_per_snr": int(c[0, abi.C_FRAMES])},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    eng.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
