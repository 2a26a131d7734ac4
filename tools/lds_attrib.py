"""LDS bank-conflict attribution of frame_sync_kernel from tools/lds_attrib.sh's PMC passes.

usage: python tools/lds_attrib.py gpurun_out/lds_attrib [--items N] [--out profiles/r05/lds/lds_attrib.json]

The FRAME_DUP_<SITE> probes were pruned from csrc/ in round 6 (profiles/r06/README.md): build the variant libraries
from a checkout of commit aec0f2e (`git worktree add /tmp/probe aec0f2e`, then tools/build_variants.py there).

Each FRAME_DUP_<SITE> variant issues one access site's LDS instructions twice (same instruction form and lane
addresses, the duplicate waited for at once; ofdm_frame.hip dup_*), so its SQ_INSTS_LDS / SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE minus the default build's are that site's instructions, conflict cycles and LDS-array cycles.
The sites' sums are compared with the kernel's totals (the remainder is everything not probed).
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

COUNTERS = ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVES")
SITES = {"dupdet": "detection register-block loads (ds_read2_b32, real + imaginary)",
         "dupmf": "matched-filter window loads (ds_read2_b32 / _b64 + b32, real + imaginary)",
         "dupcap": "capture stores (ds_write_b128)",
         "dupbp": "crossing look-ups (ds_bpermute_b32)",
         "dupcfo": "CFO / hand-off loads of fr[] (probed as ds_read2_b32)"}


def sync_counters(d: Path) -> dict:
    out = defaultdict(float)
    for f in d.glob("**/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "frame_sync_kernel" in r["Kernel_Name"]:
                out[r["Counter_Name"]] += float(r["Counter_Value"])
    return dict(out)


def main(argv):
    d = Path(argv[0])
    items = float(argv[argv.index("--items") + 1]) if "--items" in argv else 5e5 * 16
    base = sync_counters(d / "default")
    per = {c: base.get(c, 0.0) / items for c in COUNTERS[:3]}
    rows = {"kernel": {"instructions": per["SQ_INSTS_LDS"], "conflict_cycles": per["SQ_LDS_BANK_CONFLICT"],
                       "array_cycles": per["SQ_LDS_IDX_ACTIVE"],
                       "conflict_share": per["SQ_LDS_BANK_CONFLICT"] / max(per["SQ_LDS_IDX_ACTIVE"], 1e-9)}}
    print(f"frame_sync_kernel per item: {per['SQ_INSTS_LDS']:.1f} LDS instr, {per['SQ_LDS_IDX_ACTIVE']:.1f} array cycles, "
          f"{per['SQ_LDS_BANK_CONFLICT']:.1f} conflict cycles ({rows['kernel']['conflict_share']:.1%})")
    tot = defaultdict(float)
    for v, what in SITES.items():
        if not (d / v).exists():
            continue
        c = sync_counters(d / v)
        dl = {k: (c.get(k, 0.0) - base.get(k, 0.0)) / items for k in COUNTERS[:3]}
        n = max(dl["SQ_INSTS_LDS"], 1e-9)
        rows[v] = {"site": what, "instructions": dl["SQ_INSTS_LDS"], "conflict_cycles": dl["SQ_LDS_BANK_CONFLICT"],
                   "array_cycles": dl["SQ_LDS_IDX_ACTIVE"], "conflict_per_instr": dl["SQ_LDS_BANK_CONFLICT"] / n,
                   "array_per_instr": dl["SQ_LDS_IDX_ACTIVE"] / n}
        for k in ("instructions", "conflict_cycles", "array_cycles"):
            tot[k] += rows[v][k]
        print(f"  {v:7s} {dl['SQ_INSTS_LDS']:7.1f} instr  {dl['SQ_LDS_BANK_CONFLICT']:7.1f} conflict  "
              f"{dl['SQ_LDS_IDX_ACTIVE']:7.1f} array cycles  ({rows[v]['conflict_per_instr']:.2f} / "
              f"{rows[v]['array_per_instr']:.2f} per instr)  {what}")
    rows["probed_sum"] = dict(tot)
    rows["unprobed"] = {"instructions": per["SQ_INSTS_LDS"] - tot["instructions"],
                        "conflict_cycles": per["SQ_LDS_BANK_CONFLICT"] - tot["conflict_cycles"],
                        "array_cycles": per["SQ_LDS_IDX_ACTIVE"] - tot["array_cycles"]}
    print(f"  probed sum {tot['instructions']:.1f} instr, {tot['conflict_cycles']:.1f} conflict; unprobed "
          f"{rows['unprobed']['instructions']:.1f} instr, {rows['unprobed']['conflict_cycles']:.1f} conflict")
    if "--out" in argv:
        Path(argv[argv.index("--out") + 1]).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
