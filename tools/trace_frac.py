"""Roofline fraction of a bench line recomputed from a rocprofv3 kernel trace of that same bench command.

usage: python tools/trace_frac.py <trace dir> <bench json> [--clock <pmc dir>] [--out <json>]

The trace (rocprofv3 --kernel-trace) records every dispatch of the run, warm-up steps included; the bench line's
`roofline.frac` averages only its timed launches (HIP events).  This keeps the receiver dispatches of the timed
steps -- the last `steps` steps' worth of them, in dispatch order -- and prices them exactly as
bench.make_roofline does: frac = units per launch x VALU wave-instructions per unit (the line's certified
PMC record) / mean duration / nominal VALU issue peak.  With --clock, the SQ clock of a separate
`rocprofv3 --pmc GRBM_GUI_ACTIVE` run of the same command (GRBM_GUI_ACTIVE / XCDs / dispatch duration, per
receiver dispatch, timed steps only) is recorded beside it.
"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

XCDS = 8
ROOT = Path(__file__).resolve().parents[1]


def receiver_dispatches(trace_dir: Path, kernel: str) -> list[dict]:
    """dispatches of the receiver kernel(s) in dispatch order; `kernel` is bench's name, '+'-joined"""
    names = kernel.split("+")
    f = next(trace_dir.glob("**/*kernel_trace.csv"))
    rows = [r for r in csv.DictReader(open(f)) if any(n in r["Kernel_Name"] for n in names)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def split(rows: list[dict], line: dict) -> tuple[list[dict], int]:
    """(the timed steps' receiver dispatches, dispatches per timed launch): every step dispatches the same
    number of receiver kernels, the warm-up steps come first, and bench's `launches` are the timed region's
    HIP-event brackets (c3: 4 receiver launches per step; frame: one per step, i.e. two sync + symbol pairs)"""
    steps, warm, launches = line["steps"], line["warmup"], int(line["roofline"]["launches"])
    per_step = len(rows) // (steps + warm)
    assert per_step * (steps + warm) == len(rows), (len(rows), steps, warm)
    per_launch = per_step * steps // launches
    return rows[-per_step * steps:], per_launch


def launch_ns(rows: list[dict], per_launch: int) -> list[float]:
    """duration of each launch: the sum of its dispatches"""
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    return [sum(d[i:i + per_launch]) for i in range(0, len(d), per_launch)]


def clock_ghz(pmc_dir: Path, kernel: str, line: dict) -> float | None:
    """GRBM_GUI_ACTIVE / XCDs / duration over the timed receiver dispatches of a --pmc GRBM_GUI_ACTIVE run"""
    files = list(pmc_dir.glob("**/*counter_collection.csv"))
    if not files:
        return None
    names = kernel.split("+")
    rows = [r for r in csv.DictReader(open(files[0]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and any(n in r["Kernel_Name"] for n in names)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    rows, _ = split(rows, line)
    cyc = sum(float(r["Counter_Value"]) for r in rows) / XCDS
    ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    return cyc / ns if ns else None


def main(argv):
    trace_dir, bench = Path(argv[0]), Path(argv[1])
    line = json.loads(bench.read_text().strip().splitlines()[-1])
    rf = line["roofline"]
    kernel, upl, ipu = rf["kernel"], rf["units_per_launch"], rf.get("instr_per_unit")
    pmc_src = "the line's certified PMC record"
    if not ipu:       # the line predates its PMC record: take the record of the same build (same kernel id)
        wl = line["config"]["workload"]
        rec = json.loads((ROOT / "profiles" / "pmc_summary.json").read_text()).get({"c4": "c3"}.get(wl, wl), {})
        if rec.get("build_id") and rec.get("build_id") == rf.get("lib_build_id"):
            ipu = rec["valu_instr_per_unit"]
            pmc_src = f"profiles/pmc_summary.json[{wl}] (build {rec['build_id']} = the line's library)"
    rows, per_launch = split(receiver_dispatches(trace_dir, kernel), line)
    ns = launch_ns(rows, per_launch)
    avg_s = sum(ns) / len(ns) * 1e-9
    out = {"bench_line": str(bench), "trace": str(trace_dir), "kernel": kernel,
           "dispatches_in_trace": len(receiver_dispatches(trace_dir, kernel)), "timed_launches": len(ns),
           "dispatches_per_launch": per_launch,
           "trace_avg_launch_ms": avg_s * 1e3, "line_avg_launch_ms": rf["avg_launch_ms"],
           "line_frac": rf.get("frac")}
    if rf.get("bound") == "hbm":     # fft64: algorithmic bytes per unit against the HBM peak (GB/s)
        bpu = rf["algorithmic_bytes_per_unit"]
        out["bytes_per_unit"] = bpu
        out["trace_frac"] = upl * bpu / avg_s / 1e9 / rf["peak"]
        out["line_events_frac"] = upl * bpu / (rf["avg_launch_ms"] * 1e-3) / 1e9 / rf["peak"]
        out["frac_rel_diff"] = out["trace_frac"] / out["line_events_frac"] - 1
        ipu = None
    if ipu:
        out["instr_per_unit"], out["pmc_source"] = ipu, pmc_src
        out["trace_frac"] = upl * ipu / avg_s / rf["peak"]
        out["line_events_frac"] = upl * ipu / (rf["avg_launch_ms"] * 1e-3) / rf["peak"]
        out["frac_rel_diff"] = out["trace_frac"] / out["line_events_frac"] - 1
    if "--clock" in argv:
        out["clock_ghz"] = clock_ghz(Path(argv[argv.index("--clock") + 1]), kernel, line)
    text = json.dumps(out, indent=1)
    print(text)
    if "--out" in argv:
        Path(argv[argv.index("--out") + 1]).write_text(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
