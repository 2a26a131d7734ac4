"""Issue cap of the frame workload's two kernels from their gfx950 assembly, every VALU instruction classified
(no "ambiguous" class, unlike tools/mix_cap.py): each kernel's basic blocks weighted by how often a (trial, SNR)
item runs them, the one unknown weight -- the fraction u of items the lazy capture leaves undecided after its first
detection round -- fitted to the measured SQ_INSTS_VALU of the sync kernel.

usage: python tools/frame_mix.py <pmc dir>... [--items N] [--waves 3] [--record]

The assembly is compiled here from the library's sources with build_lib's flags (ofdm_frame_fix.hip for the sync
kernel, ofdm_frame_sym.hip for the symbol kernel), so run it on the tree that built the profiled library;
--record takes the build id from the PMC run's kernel_ids.json (tools/gpu_profile.sh) and stores the cap as
profiles/pmc_summary.json["frame"]["issue_model"] (method "classified") and profiles/frame_mix.json.

Sync kernel block weights per item (the fixed-geometry kernel is straight-line per phase, ofdm_frame.hip):
  * the capture-pass loop of round 0 (the first depth-2 loop holding Philox multiplies): its passes per item,
    ceil(blocks / (64 FRAME_CAP_U)) for the blocks of capture samples [0, B1 + 47) -- 2 for the reference capture;
  * the run's capture offsets (the blocks a uniform k == 0 branch skips): 1 / FRAME_ITEM_RUN;
  * the blocks skipped when round 0 decides Packet_Selection (the rest of the capture, round-1 detection, the
    undecided selection): u;
  * the matched filter's per-instant fallback (a depth-3 loop: windows that leave the capture) and the blocks
    outside the item loop: 0;
  * every other block of the item loop: 1.
Symbol kernel: its item loop's blocks once each, the class shares of that code scaled to its measured VALU count.
The classes and their SIMD cycles per wave-instruction are tools/isa_mix.py's (profiles/r01/ubench); the dynamic
class counters SQ_INSTS_VALU_{FMA,MUL,ADD}_F32 / TRANS / INT64 / CVT of the same build are printed beside the
model's, as its check.  cap = 2 (VALU_sync + VALU_sym) / (priced cycles of both): the fraction of the nominal
VALU issue peak the kernels' mix allows."""
from __future__ import annotations

import collections
import csv
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(PKG))
from isa_mix import COST, classify  # noqa: E402

SYNC = "_ZN4ofdm17frame_sync_kernelILi2ELi3008ELi12EEEvNS_9FrameArgsE"
SYM = "_ZN4ofdm16frame_sym_kernelILb0ELi2EEEvNS_9FrameArgsE"
CLASSES = ("fast", "slow", "trans", "cnd")
DYN = {"fma_f32": re.compile(r"^v_(fma|fmac|fmamk|fmaak)_f32"), "mul_f32": re.compile(r"^v_mul_f32"),
       "add_f32": re.compile(r"^v_(add|sub|subrev)_f32"), "trans": re.compile(r"^v_(log|sin|cos|sqrt|rcp|exp|rsq)_f32"),
       "int64": re.compile(r"^v_(mad_u64_u32|mad_i64_i32|lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|mov_b64)"),
       "cvt": re.compile(r"^v_cvt_")}
MEAS = {"fma_f32": "SQ_INSTS_VALU_FMA_F32", "mul_f32": "SQ_INSTS_VALU_MUL_F32", "add_f32": "SQ_INSTS_VALU_ADD_F32",
        "trans": "SQ_INSTS_VALU_TRANS_F32", "int64": "SQ_INSTS_VALU_INT64", "cvt": "SQ_INSTS_VALU_CVT"}


def asm(src: str) -> list[str]:
    from build_lib import CFLAGS, HIPCC, SOURCE_FLAGS
    s = subprocess.run([HIPCC, *CFLAGS, *SOURCE_FLAGS.get(src, []), "--cuda-device-only", "-S",
                        str(PKG / "csrc" / src), "-o", "-"], capture_output=True, text=True, check=True)
    return s.stdout.splitlines()


def blocks(lines):
    """[(name, loop depth, [(op, args)], innermost loop header)] of a kernel body (the header from LLVM's
    "in Loop: Header=BBk_n Depth=d" comments)"""
    out, cur = [], None
    for l in lines:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?(.*)", l)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2))
            h = re.search(r"Header=(\w+)", m.group(2))
            cur = [m.group(1), int(d.group(1)) if d else 0, [], h.group(1) if h else None]
            out.append(cur)
            continue
        t = l.strip().split(None, 1)
        if cur is None or not t or t[0].startswith((";", ".")):
            continue
        cur[2].append((t[0], t[1] if len(t) > 1 else ""))
    return out


def kernel_blocks(text: list[str], name: str):
    start = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
    return blocks(text[start:end])


def weights(bbs, passes0: float, run: int = 4):
    """per-item weight of each sync-kernel block as (constant, coefficient of u), u = 1 - decided"""
    label = {b[0]: i for i, b in enumerate(bbs)}

    def target(i, op):
        """index of the block the block i's branch `op` jumps to, or None"""
        t = [a for o, a in bbs[i][2] if o == op]
        return label.get(t[0].strip()) if t else None

    def back_edges(i):
        """targets of the block i's backward branches"""
        return [label[a.strip()] for o, a in bbs[i][2]
                if o.startswith(("s_branch", "s_cbranch")) and a.strip() in label and label[a.strip()] <= i]

    philox = [i for i, b in enumerate(bbs) if b[1] == 2 and sum(op == "v_mad_u64_u32" for op, _ in b[2]) >= 40]
    detect = [i for i, b in enumerate(bbs) if sum(op == "v_alignbit_b32" for op, _ in b[2]) >= 10]
    assert len(philox) == 2 and len(detect) == 2, (philox, detect)

    # the item loop: the outermost loop around the capture passes (its back edge from the last latch)
    lo, hi = min(((h, l) for l in range(philox[0], len(bbs)) for h in back_edges(l) if h <= philox[0]),
                 key=lambda hl: hl[0])
    w = {}
    for i in range(lo, hi + 1):
        w[i] = (1.0, 0.0)
        if bbs[i][1] >= 3:
            w[i] = (0.0, 0.0)                                   # per-instant matched-filter fallback
    # the run's capture offsets (k == 0, a uniform branch over the first item of each run): the item-loop block
    # holding a whole philox10 before the capture passes, and the blocks the nearest uniform branch over it skips
    pr = next(i for i in range(lo, philox[0])
              if bbs[i][1] == 1 and sum(op in ("v_mad_u64_u32", "v_mul_hi_u32") for op, _ in bbs[i][2]) >= 15)
    r0 = next(i for i in range(pr - 1, lo - 1, -1) if (target(i, "s_cbranch_scc1") or 0) > pr)
    for i in range(r0 + 1, target(r0, "s_cbranch_scc1")):
        w[i] = (1.0 / run, 0.0)
    # round 0's capture-pass loop: every block of it (the blocks LLVM annotates with its header) once per pass
    for i in range(lo, hi + 1):
        if bbs[i][3] == bbs[philox[0]][3] and bbs[i][1] == bbs[philox[0]][1]:
            w[i] = (passes0, 0.0)
    # round 0 decided: the uniform branch after the round-0 detection that jumps past round 1 and the
    # undecided Packet_Selection; every block it skips is on the undecided path
    d0 = next(i for i in range(detect[0] + 1, philox[1]) if (target(i, "s_cbranch_vccnz") or 0) > detect[1])
    for i in range(d0 + 1, target(d0, "s_cbranch_vccnz")):
        if w[i][0]:
            w[i] = (0.0, 1.0)
    # the matched filter's run is one straight-line copy per float parity of the item (ofdm_frame.hip mf_run): the two
    # copies (each opening with its run's 28 ds_read_b64) run on half the items each on average
    mf = [i for i in range(lo, hi + 1) if bbs[i][1] == 2 and sum(op == "ds_read_b64" for op, _ in bbs[i][2]) >= 20]
    if len(mf) == 2:
        join = target(mf[1] - 2, "s_branch")
        assert join and join > mf[1], (mf, join)
        for i in range(mf[0], join):
            w[i] = (0.5 * w[i][0], 0.5 * w[i][1])
    return w


def tally(bbs, w):
    """per-item class / dynamic-group / opcode counts, each as [constant, u-coefficient]"""
    cls = collections.defaultdict(lambda: [0.0, 0.0])
    dyn = collections.defaultdict(lambda: [0.0, 0.0])
    ops = collections.defaultdict(lambda: [0.0, 0.0])
    for i, (c0, c1) in w.items():
        for op, args in bbs[i][2]:
            c = classify(op, args)
            if c not in CLASSES:
                continue
            for k in (c, "valu"):
                cls[k][0] += c0; cls[k][1] += c1
            ops[(c, op)][0] += c0; ops[(c, op)][1] += c1
            for k, rx in DYN.items():
                if rx.match(op):
                    dyn[k][0] += c0; dyn[k][1] += c1
    return cls, dyn, ops


def pmc(dirs, kernel_frag):
    """counter sums over the kernel's dispatches; a counter collected in several passes is taken from the
    first pass holding it"""
    acc, seen = {}, set()
    for d in dirs:
        got = collections.defaultdict(float)
        for f in Path(d).glob("**/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if kernel_frag in r["Kernel_Name"]:
                    got[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in got.items():
            if k not in seen:
                acc[k] = v
                seen.add(k)
    return acc


def model(dirs, items: float, waves: int, sync_text=None, sym_text=None) -> dict:
    sbb = kernel_blocks(sync_text or asm("ofdm_frame_fix.hip"), SYNC)
    cls, dyn, ops = tally(sbb, weights(sbb, 2.0))
    ybb = kernel_blocks(sym_text or asm("ofdm_frame_sym.hip"), SYM)
    ycls, _, _ = tally(ybb, {i: (1.0, 0.0) for i, b in enumerate(ybb) if b[1] >= 1})
    ms, my = pmc(dirs, "frame_sync_kernel"), pmc(dirs, "frame_sym_kernel")
    v = ms["SQ_INSTS_VALU"] / items
    u = (v - cls["valu"][0]) / cls["valu"][1]
    n = {k: cls[k][0] + u * cls[k][1] for k in (*CLASSES, "valu")}
    vy = my["SQ_INSTS_VALU"] / items
    ny = {k: vy * ycls[k][0] / ycls["valu"][0] for k in CLASSES}
    cost = COST[waves]
    cyc_s = sum(cost[k] * n[k] for k in CLASSES)
    cyc_y = sum(cost[k] * ny[k] for k in CLASSES)
    return {
        "waves_per_simd": waves, "items": items, "undecided_fraction": u,
        "sync": {"kernel": SYNC, "valu_per_item": v, "classes_per_item": {k: n[k] for k in CLASSES},
                 "priced_cycles_per_item": cyc_s, "cap_frac": 2 * v / cyc_s,
                 "class_check_per_item": {k: {"model": dyn[k][0] + u * dyn[k][1], "measured": ms.get(c, float("nan")) / items}
                                          for k, c in MEAS.items()},
                 "top_ops": [(c, op, round(a + u * b, 1)) for (c, op), (a, b) in
                             sorted(ops.items(), key=lambda kv: -(kv[1][0] + u * kv[1][1]))[:25]]},
        "sym": {"kernel": SYM, "valu_per_item": vy, "classes_per_item": ny, "priced_cycles_per_item": cyc_y,
                "cap_frac": 2 * vy / cyc_y},
        "cap_frac": 2 * (v + vy) / (cyc_s + cyc_y)}


def main(argv):
    dirs = [a for a in argv if not a.startswith("--") and Path(a).is_dir()]
    waves = int(argv[argv.index("--waves") + 1]) if "--waves" in argv else 3
    if "--items" in argv:
        items = float(argv[argv.index("--items") + 1])
    else:       # the profiled bench command's (trial, SNR) items: units / data symbols per frame
        items = json.loads((ROOT / "profiles" / "pmc_summary.json").read_text())["frame"]["units_total_in_run"] / 2
    out = model(dirs, items, waves)
    print(json.dumps(out, indent=1))
    if "--record" in argv:
        ids = json.loads((Path(dirs[0]).parent / "kernel_ids.json").read_text())["ids"]
        out["build_id"] = ids["frame"]
        (ROOT / "profiles" / "frame_mix.json").write_text(json.dumps(out, indent=1) + "\n")
        p = ROOT / "profiles" / "pmc_summary.json"
        summary = json.loads(p.read_text())
        summary["frame"]["issue_model"] = {
            "build_id": ids["frame"], "waves_per_simd": waves, "cap_frac": out["cap_frac"], "method": "classified",
            "undecided_fraction": out["undecided_fraction"],
            "sync_cap_frac": out["sync"]["cap_frac"], "sym_cap_frac": out["sym"]["cap_frac"],
            "source": "tools/frame_mix.py: every VALU instruction of both kernels' gfx950 assembly classified, blocks "
                      "weighted per item (undecided fraction fitted to SQ_INSTS_VALU of %s), priced with "
                      "profiles/r01/ubench/ costs; profiles/frame_mix.json"
                      % ", ".join(str(Path(d).resolve().relative_to(ROOT)) for d in dirs)}
        p.write_text(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
