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
--split-from frame adds a point estimate inside that range: the ambiguous instructions split into fast / slow /
VCC-cndmask as in the classified model of frame's sync kernel (profiles/frame_mix.json: its per-class counts minus
the part the class counters cover), for a kernel built from the same phases (frame_sync_long_kernel).
--record stores it as pmc_summary.json[workload]["issue_model"] with the library's build id (method "dynamic", or
"dynamic_split" with the point estimate as cap_frac)."""
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


def frame_split(mix: dict) -> dict:
    """fast / slow / cnd shares of the instructions the class counters do not cover, in a classified frame_mix
    record: the sync kernel's per-class counts minus its model counts of the counter-covered groups"""
    cl, ck = mix["sync"]["classes_per_item"], mix["sync"]["class_check_per_item"]
    rest = {"fast": cl["fast"] - sum(ck[k]["model"] for k in ("fma_f32", "mul_f32", "add_f32")),
            "slow": cl["slow"] - sum(ck[k]["model"] for k in ("int64", "cvt")), "cnd": cl["cnd"]}
    tot = sum(rest.values())
    return {k: v / tot for k, v in rest.items()}


def price_split(c, waves, split):
    """the cap with the ambiguous instructions priced by the given class shares"""
    g = lambda k: c.get("SQ_INSTS_VALU_" + k, 0.0)   # noqa: E731
    valu = c["SQ_INSTS_VALU"]
    fast = g("FMA_F32") + g("MUL_F32") + g("ADD_F32")
    trans = g("TRANS_F32") + g("TRANS_F64")
    slow = g("INT64") + g("CVT") + g("FMA_F64") + g("MUL_F64") + g("ADD_F64")
    amb = valu - fast - trans - slow
    cost = COST[waves]
    cyc = (cost["fast"] * (fast + amb * split["fast"]) + cost["trans"] * trans +
           cost["slow"] * (slow + amb * split["slow"]) + cost["cnd"] * amb * split["cnd"])
    return 2 * valu / cyc


def main(argv):
    wl, waves = argv[0], int(argv[1])
    split_from = argv[argv.index("--split-from") + 1] if "--split-from" in argv else None
    dirs = [a for a in argv[2:] if not a.startswith("--") and a != split_from]
    c = counters(dirs, SETS[wl])
    lo, hi, shares = price(c, waves)
    print(f"{wl}: dynamic mix {json.dumps({k: round(v, 4) for k, v in shares.items()})}")
    print(f"  cap at {waves} waves/SIMD: {lo:.3f} (ambiguous classes slow) .. {hi:.3f} (fast) of the nominal peak")
    est = split = None
    if split_from:
        mix = json.loads((ROOT / "profiles" / f"{split_from}_mix.json").read_text())
        split = frame_split(mix)
        est = price_split(c, waves, split)
        print(f"  ambiguous split as {split_from}'s classified sync kernel {json.dumps({k: round(v, 4) for k, v in split.items()})}: "
              f"cap {est:.3f}")
    if "--record" in argv:
        ids = json.loads((Path(dirs[0]).parent / "kernel_ids.json").read_text())["ids"]
        out = ROOT / "profiles" / "pmc_summary.json"
        summary = json.loads(out.read_text())
        m = {"build_id": ids.get(wl), "waves_per_simd": waves, "cap_frac": lo, "cap_frac_range": [lo, hi],
             "dynamic_shares": shares, "method": "dynamic",
             "source": "tools/mix_cap.py: SQ_INSTS_VALU_* class counters (%s) priced with profiles/r01/ubench/ costs"
                       % ", ".join(str(Path(d).resolve().relative_to(ROOT)) for d in dirs)}
        if split:
            m.update(cap_frac=est, method="dynamic_split", ambiguous_split=split,
                     split_source=f"profiles/{split_from}_mix.json (build {mix.get('build_id')})")
        summary[wl]["issue_model"] = m
        out.write_text(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
