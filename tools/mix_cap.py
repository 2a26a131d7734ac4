"""Issue cap of a kernel from its DYNAMIC VALU mix: rocprofv3 class counters priced with the measured
per-class issue costs (profiles/r01/ubench/ubench_bank_forms.txt, the classes of tools/isa_mix.py).

usage: python tools/mix_cap.py <workload> <waves/SIMD> <pmc dir> [<pmc dir> ...] [--record]

For kernels whose loop structure tools/isa_mix.py cannot price (frame_sync_kernel: five phases of predicated
code and data-dependent trip counts).  The counters split SQ_INSTS_VALU into
  fast   SQ_INSTS_VALU_{FMA,MUL,ADD}_F32 (VGPR operands assumed)
  trans  SQ_INSTS_VALU_TRANS_F32 / _F64
  slow   SQ_INSTS_VALU_INT64 (v_mad_u64_u32), _CVT, the f64 arithmetic
  ambiguous  SQ_INSTS_VALU_INT32 and the rest (bitop3 / add_u32 are fast, shifts, alignbit, DPP, readlane slow,
             v_cndmask with VCC far slower): priced once all fast and once all slow, which bounds the cap.
cap = 2 VALU / priced SIMD cycles (the nominal peak issues one wave-instruction per 2 cycles).
--record stores it as pmc_summary.json[workload]["issue_model"] with the library's build id."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from isa_mix import COST  # noqa: E402
from pmc_summary import kernel_key  # noqa: E402

SETS = {"frame": ("frame_sync_kernel", "frame_sym_kernel"), "frame8": ("frame_sync_long_kernel", "frame_sym_kernel"),
        "c3": ("rx_pack_kernel",), "c5": ("rx_pack_kernel",), "c2": ("rx_pack_kernel",)}


def counters(dirs, kernels):
    """class counters summed over the kernels' dispatches; SQ_INSTS_VALU (in every pass) from the first dir"""
    acc = defaultdict(float)
    for i, d in enumerate(dirs):
        for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
            if kernel_key(r["Kernel_Name"]) in kernels and not (i and r["Counter_Name"] == "SQ_INSTS_VALU"):
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def price(c, waves):
    g = lambda k: c.get("SQ_INSTS_VALU_" + k, 0.0)   # noqa: E731
    valu = c["SQ_INSTS_VALU"]
    fast = g("FMA_F32") + g("MUL_F32") + g("ADD_F32")
    trans = g("TRANS_F32") + g("TRANS_F64")
    slow = g("INT64") + g("CVT") + g("FMA_F64") + g("MUL_F64") + g("ADD_F64")
    amb = valu - fast - trans - slow
    cost = COST[waves]
    lo_cyc = cost["fast"] * fast + cost["trans"] * trans + cost["slow"] * (slow + amb)     # ambiguous all slow
    hi_cyc = cost["fast"] * (fast + amb) + cost["trans"] * trans + cost["slow"] * slow     # ambiguous all fast
    shares = {k: v / valu for k, v in (("fast", fast), ("trans", trans), ("slow", slow), ("ambiguous", amb))}
    return 2 * valu / lo_cyc, 2 * valu / hi_cyc, shares


def main(argv):
    wl, waves = argv[0], int(argv[1])
    dirs = [a for a in argv[2:] if not a.startswith("--")]
    c = counters(dirs, SETS[wl])
    lo, hi, shares = price(c, waves)
    print(f"{wl}: dynamic mix {json.dumps({k: round(v, 4) for k, v in shares.items()})}")
    print(f"  cap at {waves} waves/SIMD: {lo:.3f} (ambiguous classes slow) .. {hi:.3f} (fast) of the nominal peak")
    if "--record" in argv:
        ids = json.loads((Path(dirs[0]).parent / "kernel_ids.json").read_text())["ids"]
        out = ROOT / "profiles" / "pmc_summary.json"
        summary = json.loads(out.read_text())
        summary[wl]["issue_model"] = {
            "build_id": ids.get(wl), "waves_per_simd": waves, "cap_frac": lo, "cap_frac_range": [lo, hi],
            "dynamic_shares": shares, "method": "dynamic",
            "source": "tools/mix_cap.py: SQ_INSTS_VALU_* class counters (%s) priced with profiles/r01/ubench/ costs"
                      % ", ".join(str(Path(d).resolve().relative_to(ROOT)) for d in dirs)}
        out.write_text(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
