"""Summarise rocprofv3 --kernel-trace / --pmc runs (tools/gpu_profile.sh) into profiles/.

usage: python tools/pmc_summary.py <gpurun_out dir> <workload> <units_total_in_run> [--out FILE]

<units_total_in_run>: symbol-SNR evaluations the profiled command processed in ALL its receiver
dispatches (warmup steps included), e.g. (warmup + steps) x symbols x 16 SNR points.

Counters are summed over every dispatch of the workload's receiver kernels (symbol mode:
rx_pack_kernel (real AWGN) / rx_ls_kernel / rx_ideal_kernel; frame mode: frame_sync_kernel + frame_sym_kernel, which the frame
timer brackets together) and divided by the units:
  * HBM bytes: FETCH_SIZE (KB) x 1024 x 2 -- gfx950 reports half of the bytes of wide (16 B/lane)
    coalesced streaming reads, LDS-DMA included (MI355X_MICROARCH.md, HBM section) -- plus
    WRITE_SIZE (KB) x 1024;
  * VALU: SQ_INSTS_VALU wave-instructions per unit, and the issue rate against the peak
    (256 CUs x 4 SIMDs x 1 wave-instruction / 2 cycles) at 2.4 GHz and at the clock
    GRBM_GUI_ACTIVE / duration shows.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KERNELS = ("rx_pack_kernel", "rx_ls_kernel", "rx_ideal_kernel", "tx_symbols_kernel", "frame_sync_long_kernel",
           "frame_sync_kernel", "frame_sym_kernel", "fft64_lds_kernel")
RX_SETS = (("rx_pack_kernel",), ("rx_ls_kernel",), ("rx_ideal_kernel",), ("frame_sync_long_kernel", "frame_sym_kernel"),
           ("frame_sync_kernel", "frame_sym_kernel"), ("fft64_lds_kernel",))
CUS, SIMDS, XCDS = 256, 4, 8
NOMINAL_CLOCK = 2.4e9


def kernel_key(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def read_counters(d: Path):
    """kernel -> counter -> sum over dispatches (and dispatch counts); a counter collected in several passes
    (SQ_INSTS_VALU beside each class group) is taken from the first pass that holds it (pmc_1, pmc_2, ...)"""
    sums = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    passes = sorted(d.glob("pmc_*/"), key=lambda p: int(p.name.split("_")[1]) if p.name.split("_")[1].isdigit() else 0)
    for p in passes:
        got = defaultdict(lambda: defaultdict(float))
        cnt = defaultdict(lambda: defaultdict(int))
        for f in sorted(p.glob("**/*counter_collection.csv")):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = kernel_key(r["Kernel_Name"])
                    if not k:
                        continue
                    got[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    cnt[k][r["Counter_Name"]] += 1
        for k, cs in got.items():
            for c, v in cs.items():
                if c not in sums[k]:
                    sums[k][c], n[k][c] = v, cnt[k][c]
    return sums, n


def read_trace(d: Path):
    """Per-kernel calls / total / mean duration of the pmc_trace run: from rocprofv3's --stats summary, or, where
    a record keeps only the kernel trace, summed from its dispatch rows."""
    out = {}

    def add(name, calls, ns):
        k = kernel_key(name)
        if k:       # several instantiations of one kernel (fft64: forward and inverse) are summed
            e = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
            e["calls"] += calls
            e["total_ns"] += ns
            e["avg_ns"] = e["total_ns"] / e["calls"]

    stats = sorted(d.glob("pmc_trace/**/*kernel_stats.csv"))
    for f in stats:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                add(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]))
    if not stats:
        for f in sorted(d.glob("pmc_trace/**/*kernel_trace.csv")):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    add(r["Kernel_Name"], 1, float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out


def main(argv):
    d, workload, units = Path(argv[0]), argv[1], float(argv[2])
    out = Path(argv[argv.index("--out") + 1]) if "--out" in argv else ROOT / "profiles" / "pmc_summary.json"
    sums, ndisp = read_counters(d)
    trace = read_trace(d)
    summary = json.loads(out.read_text()) if out.exists() else {}
    rx = next(s for s in RX_SETS if s[0] in sums)
    c = defaultdict(float)
    for k in rx:
        for name, v in sums[k].items():
            c[name] += v
    t_total = sum(trace.get(k, {}).get("total_ns", 0.0) for k in rx) * 1e-9
    rd = 2.0 * c.get("FETCH_SIZE", float("nan")) * 1024
    wr = c.get("WRITE_SIZE", float("nan")) * 1024
    clk = c.get("GRBM_GUI_ACTIVE", float("nan")) / XCDS / t_total if t_total else float("nan")
    valu = c.get("SQ_INSTS_VALU", float("nan"))
    peak = CUS * SIMDS * 0.5 * NOMINAL_CLOCK
    entry = {
        "kernels": list(rx),
        "units_total_in_run": units,
        "kernel_time_s_trace": t_total,
        "hbm_read_bytes_per_unit": rd / units,
        "hbm_write_bytes_per_unit": wr / units,
        "hbm_bytes_per_unit": (rd + wr) / units,
        "hbm_gbs_measured": (rd + wr) / t_total / 1e9 if t_total else None,
        "clock_ghz": clk / 1e9,
        "valu_instr_per_unit": valu / units,
        "valu_instr_per_s": valu / t_total if t_total else None,
        "valu_issue_peak_per_s": peak,
        "valu_frac": valu / t_total / peak if t_total else None,
        "valu_frac_at_measured_clock": valu / t_total / (CUS * SIMDS * 0.5 * clk) if t_total else None,
        "counters_sum_per_unit": {k: v / units for k, v in c.items()},
        "dispatches_per_counter": {k: dict(v) for k, v in ndisp.items() if k in rx},
        "trace": trace,
        "note": "FETCH_SIZE doubled (gfx950 reports half of wide streaming reads); sums over dispatches / units",
    }
    # the build id of the kernels measured: from the session's own kernel_ids.json (tools/gpu_profile.sh, written
    # on the box from the library it profiled); bench.py refuses the record for any other build
    ids_file = d / "kernel_ids.json"
    if ids_file.exists():
        entry["build_id"] = json.loads(ids_file.read_text())["ids"].get(workload)
        entry["build_id_source"] = str(ids_file.relative_to(ROOT) if ids_file.is_relative_to(ROOT) else ids_file)
    else:
        sys.path.insert(0, str(ROOT / "tools"))
        from kernel_ids import ids  # noqa: PLC0415
        entry["build_id"] = ids()["ids"].get(workload)
        entry["build_id_source"] = "in-tree library at summary time (no kernel_ids.json in the session)"
    old = summary.get(workload, {}).get("issue_model")
    if old and old.get("build_id") == entry["build_id"]:     # tools/isa_mix.py --record: a static-code figure
        entry["issue_model"] = old
    summary[workload] = entry
    out.write_text(json.dumps(summary, indent=1, sort_keys=True))
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
