"""Summarise rocprofv3 --kernel-trace / --pmc runs (tools/gpu_profile.sh) into profiles/.

usage: python tools/pmc_summary.py <gpurun_out dir> <workload> <units_per_launch> [--out profiles/pmc_summary.json]

Per receiver launch (mean over the dispatches of the run):
  * HBM bytes: FETCH_SIZE (KB) x 1024 x 2 -- gfx950 reports half of the bytes of wide (16 B/lane)
    coalesced streaming reads, LDS-DMA included (MI355X_MICROARCH.md, HBM section) -- plus
    WRITE_SIZE (KB) x 1024;
  * VALU: SQ_INSTS_VALU wave-instructions per launch and per second against the issue peak
    (256 CUs x 4 SIMDs x 1 wave-instruction / 2 cycles, tools/ubench_valu.hip) at the clock
    GRBM_GUI_ACTIVE / duration shows.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KERNELS = ("rx_ls_kernel", "rx_ideal_kernel", "tx_symbols_kernel", "frame_sync_kernel", "frame_sym_kernel")
BYTES_PER_UNIT = 652
CUS, SIMDS, XCDS = 256, 4, 8
NOMINAL_CLOCK = 2.4e9


def kernel_key(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def read_counters(d: Path):
    vals = defaultdict(lambda: defaultdict(list))      # kernel -> counter -> [per dispatch]
    durs = defaultdict(list)
    for f in sorted(d.glob("pmc_*/**/*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = kernel_key(r["Kernel_Name"])
                if not k:
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, durs


def read_trace(d: Path):
    out = {}
    for f in sorted(d.glob("pmc_trace/**/*kernel_stats.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = kernel_key(r["Name"])
                if k:
                    out[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    return out


def main(argv):
    d, workload, units = Path(argv[0]), argv[1], float(argv[2])
    out = Path(argv[argv.index("--out") + 1]) if "--out" in argv else ROOT / "profiles" / "pmc_summary.json"
    vals, _ = read_counters(d)
    trace = read_trace(d)
    summary = json.loads(out.read_text()) if out.exists() else {}
    # the receiver kernel of this run (symbol-mode LS / ideal, or frame mode)
    rx = next(k for k in ("rx_ls_kernel", "rx_ideal_kernel", "frame_sync_kernel") if k in vals)
    c = {k: statistics.mean(v) for k, v in vals[rx].items()}
    t = trace.get(rx, {}).get("avg_ns", float("nan")) * 1e-9
    rd = 2.0 * c.get("FETCH_SIZE", float("nan")) * 1024
    wr = c.get("WRITE_SIZE", float("nan")) * 1024
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs
    clk = c.get("GRBM_GUI_ACTIVE", float("nan")) / XCDS / t if t == t else float("nan")
    valu = c.get("SQ_INSTS_VALU", float("nan"))
    peak_valu = CUS * SIMDS * 0.5 * NOMINAL_CLOCK      # 1 wave64 VALU instruction / 2 cycles / SIMD
    entry = {
        "kernel": rx,
        "units_per_launch": units,
        "avg_launch_ms_trace": t * 1e3,
        "algorithmic_bytes_per_launch": BYTES_PER_UNIT * units,
        "fetch_size_kb_raw": c.get("FETCH_SIZE"),
        "write_size_kb_raw": c.get("WRITE_SIZE"),
        "rx_hbm_read_bytes_per_launch": rd,
        "rx_hbm_write_bytes_per_launch": wr,
        "rx_hbm_bytes_per_launch": rd + wr,
        "hbm_gbs_measured": (rd + wr) / t / 1e9,
        "clock_ghz": clk / 1e9,
        "valu_instr_per_launch": valu,
        "valu_instr_per_unit": valu / units,
        "valu_instr_per_s": valu / t,
        "valu_issue_peak_per_s": peak_valu,
        "valu_frac": valu / t / peak_valu,
        "valu_frac_at_measured_clock": valu / t / (CUS * SIMDS * 0.5 * clk),
        "counters_mean_per_launch": c,
        "trace": trace,
        "note": "FETCH_SIZE doubled (gfx950 reports half of wide streaming reads); per-dispatch means",
    }
    summary[workload] = entry
    out.write_text(json.dumps(summary, indent=1, sort_keys=True))
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
