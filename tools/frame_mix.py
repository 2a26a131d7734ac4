"""Issue cap of the frame sync kernel from its gfx950 assembly, every VALU instruction classified (no
"ambiguous" class): the kernel's basic blocks weighted by how often a (trial, SNR) item runs them, the one unknown
weight -- the fraction of items the lazy capture decides in its first detection round -- fitted to the measured
SQ_INSTS_VALU of the sync kernel.

usage: python tools/frame_mix.py <asm.s> <mangled kernel> <pmc dir>... [--waves 3] [--record]

Block weights per item (the fixed-geometry kernel's code is straight-line per phase, ofdm_frame.hip):
  * the capture-pass loop of round 0 (the first depth-2 loop holding Philox multiplies): its passes per item, i.e.
    ceil(blocks / (64 FRAME_CAP_U)) for the blocks of capture samples [0, B1 + 47) -- 2 for the reference capture;
  * the second such loop (the rest of the capture) and the second detection round (the second large block with
    v_alignbit): 1 - decided, once;
  * the matched filter's per-instant fallback (a depth-3 loop: windows that leave the capture) and the blocks
    outside the item loop: 0;
  * every other block of the item loop: 1.
The classes and their SIMD cycles per wave-instruction are tools/isa_mix.py's (profiles/r01/ubench); the dynamic
class counters SQ_INSTS_VALU_{FMA,MUL,ADD}_F32 / TRANS / INT64 / CVT of the same build (the PMC dirs) are
printed beside the model's, as its check."""
from __future__ import annotations

import collections
import csv
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from isa_mix import COST, classify  # noqa: E402

DYN = {"fma_f32": re.compile(r"^v_(fma|fmac|fmamk|fmaak)_f32"), "mul_f32": re.compile(r"^v_mul_f32"),
       "add_f32": re.compile(r"^v_(add|sub|subrev)_f32"), "trans": re.compile(r"^v_(log|sin|cos|sqrt|rcp|exp|rsq)_f32"),
       "int64": re.compile(r"^v_(mad_u64_u32|mad_i64_i32|lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|mov_b64)"),
       "cvt": re.compile(r"^v_cvt_")}


def blocks(lines):
    """[(name, loop depth, [(op, args)])] of the kernel body"""
    out, cur = [], None
    for l in lines:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?(.*)", l)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2))
            cur = [m.group(1), int(d.group(1)) if d else 0, []]
            out.append(cur)
            continue
        t = l.strip().split(None, 1)
        if cur is None or not t or t[0].startswith((";", ".")):
            continue
        cur[2].append((t[0], t[1] if len(t) > 1 else ""))
    return out


def weights(bbs, passes0: float):
    """per-item weight of each block as a function of u = 1 - decided: (constant, coefficient of u)"""
    # the blocks inside the item loop: those between the first and the last depth >= 1 block
    inner = [i for i, b in enumerate(bbs) if b[1] >= 1]
    lo, hi = inner[0], inner[-1]
    philox = [i for i in range(lo, hi + 1) if bbs[i][1] == 2 and sum(op == "v_mad_u64_u32" for op, _ in bbs[i][2]) >= 40]
    detect = [i for i in range(lo, hi + 1) if sum(op == "v_alignbit_b32" for op, _ in bbs[i][2]) >= 10]
    assert len(philox) == 2 and len(detect) == 2, (philox, detect)
    w = {}
    for i in range(lo, hi + 1):
        w[i] = (1.0, 0.0)
        if bbs[i][1] >= 3:
            w[i] = (0.0, 0.0)                                   # per-instant matched-filter fallback
    w[philox[0]] = (passes0, 0.0)
    w[philox[1]] = (0.0, 1.0)
    w[detect[1]] = (0.0, 1.0)
    # the blocks between the round-0 decision and the end of round 1 belong to the undecided path
    for i in range(philox[1], detect[1] + 1):
        if i not in (philox[1], detect[1]) and bbs[i][1] == 1:
            w[i] = (0.0, 1.0)
    return w


def pmc(dirs, kernel_frag):
    acc = collections.defaultdict(float)
    for d in dirs:
        for f in Path(d).glob("**/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if kernel_frag in r["Kernel_Name"]:
                    acc[r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def main(argv):
    path, name = argv[0], argv[1]
    dirs = [a for a in argv[2:] if not a.startswith("--") and not a.isdigit()]
    waves = int(argv[argv.index("--waves") + 1]) if "--waves" in argv else 3
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
    bbs = blocks(text[start:end])
    w = weights(bbs, 2.0)
    # per-item counts as (constant, u-coefficient) per class and per dynamic counter group
    cls = collections.defaultdict(lambda: [0.0, 0.0])
    dyn = collections.defaultdict(lambda: [0.0, 0.0])
    ops = collections.defaultdict(lambda: [0.0, 0.0])
    for i, (c0, c1) in w.items():
        for op, args in bbs[i][2]:
            c = classify(op, args)
            if c not in ("fast", "slow", "trans", "cnd"):
                continue
            for k in (c, "valu"):
                cls[k][0] += c0; cls[k][1] += c1
            ops[(c, op)][0] += c0; ops[(c, op)][1] += c1
            for k, rx in DYN.items():
                if rx.match(op):
                    dyn[k][0] += c0; dyn[k][1] += c1
    # measured: the sync kernel's counters per item (items = the PMC run's units / 2 data symbols)
    m = pmc(dirs, "frame_sync_kernel")
    items = float(next(a for a in argv if a.isdigit())) if any(a.isdigit() for a in argv[2:]) else None
    out = {"kernel": name, "waves_per_simd": waves}
    if items and m.get("SQ_INSTS_VALU"):
        v = m["SQ_INSTS_VALU"] / items
        u = (v - cls["valu"][0]) / cls["valu"][1]
        out.update(measured_valu_per_item=v, undecided_fraction=u)
        meas = {"fma_f32": "SQ_INSTS_VALU_FMA_F32", "mul_f32": "SQ_INSTS_VALU_MUL_F32", "add_f32": "SQ_INSTS_VALU_ADD_F32",
                "trans": "SQ_INSTS_VALU_TRANS_F32", "int64": "SQ_INSTS_VALU_INT64", "cvt": "SQ_INSTS_VALU_CVT"}
        out["class_check_per_item"] = {k: {"model": dyn[k][0] + u * dyn[k][1],
                                           "measured": m.get(c, float("nan")) / items} for k, c in meas.items()}
    else:
        u = 0.3
        out["undecided_fraction"] = u
        out["note"] = "no PMC data: undecided fraction assumed"
    n = {k: cls[k][0] + u * cls[k][1] for k in ("fast", "slow", "trans", "cnd", "valu")}
    cyc = sum(COST[waves][k] * n[k] for k in ("fast", "slow", "trans", "cnd"))
    out.update(model_valu_per_item=n["valu"], classes_per_item={k: n[k] for k in ("fast", "slow", "trans", "cnd")},
               priced_cycles_per_item=cyc, cap_frac=2 * n["valu"] / cyc,
               top_ops=[(c, op, round(a + u * b, 1)) for (c, op), (a, b) in
                        sorted(ops.items(), key=lambda kv: -(kv[1][0] + u * kv[1][1]))[:25]])
    print(json.dumps(out, indent=1))
    if "--record" in argv:
        o = ROOT / "profiles" / "frame_mix.json"
        o.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
