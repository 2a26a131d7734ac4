#!/usr/bin/env python3
"""Classified issue cap of the frame8 workload (frame_sync_long_kernel + frame_sym_kernel<false, 0>), VERDICT r5
item 3: every VALU instruction of the long kernel's gfx950 code classified (tools/isa_mix.py classes and costs) and
weighted by how often a (trial, SNR) item executes it.

usage: python tools/frame8_mix.py <pmc dir>... [--items N] [--waves 3,3,3,3] [--record]

frame_mix.py (the reference frame's sync kernel) finds its phases by code patterns; the long kernel's 1,500 blocks
(four capture call sites, three detection rounds, unrolled matched-filter passes with their per-instant fallbacks)
are attributed by their SOURCE instead.  The library's TU is compiled once more with -g (same flags; the
instruction stream differs from the product build by a few instructions, printed as `g_build_instr_delta`), and
each instruction is mapped to the kernel-body statement it comes from: the DW_AT_call_line of the outermost
inlined call holding it (capture_blocks, the detect / select lambdas, ...), else its own line.  Weights per item:
  * outside the item loop: 0;
  * the undecided path (`if (cand == 0x7fffffff)`: round 2's piece and detection, the selection over three rounds): u;
  * the matched-filter window's missing end generated (the capture ring does not hold all of it): g;
  * the per-instant matched-filter path (windows leaving the capture): 0, its per-pass skeleton 1/3 (pass 2's
    lanes past the 137 runs take it);
  * a capture call site's pass loop: piece(0), piece(1), piece(2) 2 passes per item (a round's 2,031 samples: <= 509
    Philox blocks, 256 per pass), times the call site's weight; the window's missing end: the fixture's whole passes
    per item (regen_full) in its loop, and its last pass of 3 / 2 / 1 blocks per lane at the fixture's rates;
  * the hand-off loop: 1 + n_data = 9 iterations;
  * every other instruction of the item loop: 1.
g is the fraction tests/golden/frame8_path_rates.json records for the bench grid (a CPU simulation of the kernel's
rules on the oracle's captures); u is fitted to the measured FMA count of the sync kernel (PMC run of the same build;
v_fma / v_fmac are unambiguous) and printed beside the simulation's 1 - decided and the u the total VALU count would
give.  The sync kernel's issue classes: the instructions the SQ_INSTS_VALU_* class counters cover as MEASURED, the
rest (a third) split into fast / slow / cndmask as the weighted assembly splits its own uncovered instructions.  The
symbol kernel's classes are its item loop's, scaled to its measured VALU count.  cap = 2 (VALU_sync + VALU_sym) /
priced SIMD cycles of both.
--record stores it as profiles/pmc_summary.json["frame8"]["issue_model"] (method "classified") and
profiles/frame8_mix.json.
"""
from __future__ import annotations

import bisect
import collections
import csv
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"
SRC = PKG / "csrc" / "ofdm_frame.hip"
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(PKG))
from isa_mix import COST, classify  # noqa: E402
import frame_mix  # noqa: E402

LONG = "_ZN4ofdm22frame_sync_long_kernelILi12EEEvNS_9FrameArgsE"
SYM = "_ZN4ofdm16frame_sym_kernelILb0ELi0EEEvNS_9FrameArgsE"
CLASSES = ("fast", "slow", "trans", "cnd")
LLVM = Path("/opt/rocm/lib/llvm/bin")
FRAME_FILE = 1          # ofdm_frame.hip's index in the TU's line table (file 0 is ofdm_frame_long.hip itself)


def compile_obj(tu: str, debug: bool, out: Path) -> Path:
    from build_lib import CFLAGS, HIPCC, SOURCE_FLAGS  # noqa: PLC0415
    cmd = [HIPCC, *CFLAGS, *SOURCE_FLAGS.get(tu, []), "--cuda-device-only", "--no-gpu-bundle-output", "-c",
           *(["-g"] if debug else []), str(PKG / "csrc" / tu), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def disasm(obj: Path, sym: str) -> list[tuple[int, str, str]]:
    """[(address, mnemonic, operands)] of one kernel"""
    txt = subprocess.run([str(LLVM / "llvm-objdump"), "-d", f"--disassemble-symbols={sym}", str(obj)],
                         capture_output=True, text=True, check=True).stdout
    out = []
    for ln in txt.splitlines():
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(<\S+>)?", ln)
        if m:
            out.append((int(m.group(3), 16), m.group(1), m.group(2) + (" " + m.group(4) if m.group(4) else "")))
    return out


def inline_sites(obj: Path, kernel_pc: int) -> list[tuple[int, int, int, int]]:
    """[(lo, hi, call_line, nesting depth)] address ranges of every inlined call in the kernel's body"""
    txt = subprocess.run([str(LLVM / "llvm-dwarfdump"), "--debug-info", str(obj)], capture_output=True, text=True,
                         check=True).stdout
    dies, cur = [], None
    for ln in txt.splitlines():
        m = re.match(r"^0x[0-9a-f]+:(\s+)DW_TAG_(\w+)", ln)
        if m:
            cur = {"depth": len(m.group(1)), "tag": m.group(2), "ranges": [], "call_line": None, "low": None,
                   "call_file": None}
            dies.append(cur)
            continue
        if cur is None:
            continue
        r = re.search(r"\[0x([0-9a-f]+), 0x([0-9a-f]+)\)", ln)
        if r and "DW_OP" not in ln:
            cur["ranges"].append((int(r.group(1), 16), int(r.group(2), 16)))
        m = re.search(r"DW_AT_low_pc\s+\(0x([0-9a-f]+)\)", ln)
        if m:
            cur["low"] = int(m.group(1), 16)
        m = re.search(r"DW_AT_high_pc\s+\(0x([0-9a-f]+)\)", ln)
        if m and cur["low"] is not None:
            cur["ranges"].append((cur["low"], int(m.group(1), 16)))
        m = re.search(r"DW_AT_call_line\s+\((\d+)\)", ln)
        if m:
            cur["call_line"] = int(m.group(1))
        m = re.search(r'DW_AT_call_file\s+\("([^"]+)"\)', ln)
        if m:
            cur["call_file"] = m.group(1)
    k = next(i for i, d in enumerate(dies) if d["tag"] == "subprogram" and d["low"] == kernel_pc)
    base = dies[k]["depth"]
    sites, stack = [], []                                   # stack: depths of the enclosing inlined DIEs
    for d in dies[k + 1:]:
        if d["depth"] <= base:
            break
        while stack and stack[-1] >= d["depth"]:
            stack.pop()
        if d["tag"] == "inlined_subroutine":
            # call lines in ofdm_frame.hip only (static_for / helper bodies live in other files): 0 elsewhere
            cl = d["call_line"] if (d["call_file"] or "").endswith(SRC.name) else 0
            sites += [(lo, hi, cl, len(stack)) for lo, hi in d["ranges"]]
            stack.append(d["depth"])
    return sites


def line_table(obj: Path) -> tuple[list[int], list[tuple[int, int]]]:
    """sorted row addresses and their (file index, line)"""
    txt = subprocess.run([str(LLVM / "llvm-dwarfdump"), "--debug-line", str(obj)], capture_output=True, text=True,
                         check=True).stdout
    rows = []
    for ln in txt.splitlines():
        m = re.match(r"^0x([0-9a-f]{16})\s+(\d+)\s+(\d+)\s+(\d+)", ln)
        if m:
            rows.append((int(m.group(1), 16), int(m.group(4)), int(m.group(2))))
    rows.sort()
    return [r[0] for r in rows], [(r[1], r[2]) for r in rows]


def src_line(text: list[str], needle: str, start: int = 0) -> int:
    """1-based line of the first source line at or after `start` containing `needle`"""
    return next(i + 1 for i in range(start, len(text)) if needle in text[i])


def anchors() -> dict:
    t = SRC.read_text().splitlines()
    k = src_line(t, "void frame_sync_long_kernel(FrameArgs a)") - 1
    a = {"kernel": k + 1,
         "item_for": src_line(t, "for (int64_t i = run_end - FRAME_ITEM_RUN; i < a.n_items;) {", k),
         "piece0": src_line(t, "piece(0);", k),
         "piece1": src_line(t, "piece(1);", k),
         "undec_lo": src_line(t, "if (cand == 0x7fffffff) {", k),
         "undec_hi": src_line(t, "const bool sync_fail = cand == 0x7fffffff;", k),
         "regen_lo": src_line(t, "if (hi >= res_hi || lo < res_lo) {", k),
         "fb_lo": src_line(t, "// the per-instant path (windows leaving the capture)", k),
         "fb_inner_lo": src_line(t, "if (n >= L + 20) {", k),
         "handoff_lo": src_line(t, "for (int j = lx; j < 64 * nw; j += 64) {", k),
         "handoff_hi": src_line(t, "dst[win_off(n, a.ipb, nw) + w] = v;", k)}
    a["regen_gen"] = src_line(t, "gen(fwd ? max(lo, res_hi) : lo, fwd ? hi + 1 : min(hi + 1, res_lo), std::true_type{});",
                              a["regen_lo"] - 1)
    a["regen_hi"] = a["regen_gen"] + 2
    a["fb_inner_hi"] = src_line(t, "v.y = fmaf(xi, h, v.y);", a["fb_inner_lo"] - 1)
    a["fb_hi"] = src_line(t, "mfo[pi][o] = v;", a["fb_inner_hi"] - 1)
    a["item_end"] = src_line(t, "// the next capture overwrites this item's region", a["handoff_hi"] - 1)
    a["undec_capture"] = src_line(t, "piece(2);", a["undec_lo"] - 1)
    # capture_blocks<..., TRIM = true>'s last pass (the window's missing end): 3, 2 or 1 blocks per lane
    cb = src_line(t, "__device__ __forceinline__ void capture_blocks(")
    for u in (3, 2, 1):
        a[f"tail{u}"] = src_line(t, f"pass(std::integral_constant<int, {u}>{{}}, p0);", cb)
    return a


def loops(ins) -> list[tuple[int, int]]:
    """(header address, latch address) of every backward branch"""
    out = []
    for addr, op, args in ins:
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.search(r"<\S+\+0x([0-9a-f]+)>", args)
            if m:
                tgt = int(m.group(1), 16) + ins[0][0]
                if tgt <= addr:
                    out.append((tgt, addr))
    return out


def chains(ins, sites, rows) -> dict:
    """address -> the statement lines of its inlining chain, outermost call first, its own line last"""
    ra, rv = rows
    by_depth = collections.defaultdict(list)
    for lo, hi, cl, dep in sites:
        by_depth[dep].append((lo, hi, cl))
    for v in by_depth.values():
        v.sort()
    out = {}
    prev = []
    for addr, _, _ in ins:
        ch = []
        for dep in sorted(by_depth):
            v = by_depth[dep]
            i = bisect.bisect_right(v, (addr, float("inf"), 0)) - 1
            while i >= 0 and v[i][0] <= addr:
                if addr < v[i][1]:
                    ch.append(v[i][2])
                    break
                i -= 1
        j = bisect.bisect_right(ra, addr) - 1
        own = rv[j][1] if j >= 0 and rv[j][0] == FRAME_FILE else 0
        ch = [x for x in ch if x]
        if own:
            ch.append(own)
        elif j >= 0 and rv[j] == (FRAME_FILE, 0) and prev[:len(ch)] == ch:
            ch = prev                        # an artificial (line 0) instruction: the statement it follows
        out[addr] = ch
        prev = ch
    return out


def weights(ins, sites, rows, a, rates: dict, nw: int):
    """per-instruction weight as (constant, coefficient of u) -- the fixture's regeneration rates enter the constant:
    the items generating the missing end of their matched-filter window, their whole passes and their last pass's
    width"""
    g = rates["regen"]
    tails = {u: rates[f"regen_tail{u}"] for u in (3, 2, 1)}
    ch = chains(ins, sites, rows)
    lp = loops(ins)
    item = max(lp, key=lambda l: l[1] - l[0])
    # a Philox capture loop: the smallest loop around a capture pass (>= 40 v_mad_u64_u32), at most 8 KB of code
    phil = [l for l in lp if l[1] - l[0] < 0x2000
            and sum(1 for x, op, _ in ins if l[0] <= x <= l[1] and op == "v_mad_u64_u32") >= 40]
    inner_loops = [l for l in lp if l != item and l[1] - l[0] < 0x2000]

    def within(c, lo, hi):
        return any(lo <= x <= hi for x in c)

    w = {}
    for addr, op, args in ins:
        c_ = ch[addr]
        # the item loop by source (the compiler places some of its blocks past the loop's latch): its statements
        if not within(c_[:1], a["item_for"], a["item_end"]):
            w[addr] = (0.0, 0.0)
            continue
        c, cu = 1.0, 0.0
        tail = None
        if within(c_, a["undec_lo"], a["undec_hi"] - 1):
            c, cu = 0.0, 1.0
        elif within(c_, a["regen_lo"], a["regen_hi"] + 1):
            c = g
            tail = next((u for u in (3, 2, 1) if a[f"tail{u}"] in c_), None)
            if tail is not None:                    # a last pass of `tail` blocks per lane: tails[tail] of the items
                c = tails[tail]
        elif within(c_, a["fb_inner_lo"], a["fb_inner_hi"] + 2):
            c = 0.0
        elif within(c_, a["fb_lo"], a["fb_hi"]):
            c = 1.0 / 3.0
        mult = 1.0
        if tail is None and any(l[0] <= addr <= l[1] for l in phil):
            sites_ = (a["piece0"], a["piece1"], a["undec_capture"], a["regen_gen"])
            site = next((x for x in c_ if x in sites_), None)
            # a round's piece: 2,031 samples, <= 509 Philox blocks = 2 passes of 256; the window's missing end: its whole
            # passes per item over the g items that generate it
            mult = (1.0 if site is None else (rates["regen_full"] / g if g else 0.0) if site == a["regen_gen"]
                    else 2.0)
        elif within(c_, a["handoff_lo"], a["handoff_hi"]) and any(l[0] <= addr <= l[1] for l in inner_loops):
            mult = float(nw)
        w[addr] = (c * mult, cu * mult)
    return w, item, phil


def tally(ins, w):
    cls = collections.defaultdict(lambda: [0.0, 0.0])
    for addr, op, args in ins:
        c = classify(op, args)
        if c in CLASSES:
            for k in (c, "valu"):
                cls[k][0] += w[addr][0]
                cls[k][1] += w[addr][1]
    return cls


def model(dirs, items: float, waves="3,3,3,3") -> dict:
    rates = json.loads((ROOT / "tests" / "golden" / "frame8_path_rates.json").read_text())
    g, u_sim = rates["grid_mean"]["regen"], 1.0 - rates["grid_mean"]["decided"]
    a = anchors()
    with tempfile.TemporaryDirectory() as td:
        og = compile_obj("ofdm_frame_long.hip", True, Path(td) / "long_g.o")
        on = compile_obj("ofdm_frame_long.hip", False, Path(td) / "long.o")
        ins = disasm(og, LONG)
        n_plain = len(disasm(on, LONG))
        sites = inline_sites(og, ins[0][0])
        rows = line_table(og)
    w, item, phil = weights(ins, sites, rows, a, rates["grid_mean"], 9)
    ms, my = frame_mix.pmc(dirs, "frame_sync_long_kernel"), frame_mix.pmc(dirs, "frame_sym_kernel")
    meas = {k: ms[c] / items for k, c in frame_mix.MEAS.items()}
    v = ms["SQ_INSTS_VALU"] / items

    def dyn(rx):
        return (sum(w[x][0] for x, op, _ in ins if rx.match(op)), sum(w[x][1] for x, op, _ in ins if rx.match(op)))
    # u from the FMA count: v_fma / v_fmac are unambiguous and 38 % of the kernel's VALU (the total also holds the
    # integer / move / compare instructions no class counter covers, the model's least certain part)
    f0, f1 = dyn(frame_mix.DYN["fma_f32"])
    u = (meas["fma_f32"] - f0) / f1
    cls = tally(ins, w)
    u_total = (v - cls["valu"][0]) / cls["valu"][1]
    # the instructions the class counters cover are taken as MEASURED; the rest (v - covered) is split into the
    # issue classes as the weighted assembly splits its own uncovered instructions
    covered = sum(meas.values())
    unc = collections.defaultdict(float)
    for x, op, args in ins:
        c = classify(op, args)
        if c in CLASSES and not any(rx.match(op) for rx in frame_mix.DYN.values()):
            unc[c] += w[x][0] + u * w[x][1]
    ut = sum(unc.values())
    share = {k: unc[k] / ut for k in CLASSES}
    n = {"fast": meas["fma_f32"] + meas["mul_f32"] + meas["add_f32"] + (v - covered) * share["fast"],
         "trans": meas["trans"] + (v - covered) * share["trans"],
         "slow": meas["int64"] + meas["cvt"] + (v - covered) * share["slow"],
         "cnd": (v - covered) * share["cnd"]}
    ybb = frame_mix.kernel_blocks(frame_mix.asm("ofdm_frame_sym.hip"), SYM)
    ycls, _, _ = frame_mix.tally(ybb, {i: (1.0, 0.0) for i, b in enumerate(ybb) if b[1] >= 1})
    vy = my["SQ_INSTS_VALU"] / items
    ny = {k: vy * ycls[k][0] / ycls["valu"][0] for k in CLASSES}
    # waves: the sync kernel's waves on each of a CU's four SIMDs (12-wave blocks, one per CU: 3 each; the 9-wave build
    # ran 3, 2, 2, 2).  Items are handed out dynamically, so the chip's cap is the mean of the SIMDs' caps; the symbol
    # kernel runs 3 per SIMD
    simds = [int(x) for x in str(waves).split(",")]
    cyc_y = sum(COST[3][k] * ny[k] for k in CLASSES)          # the symbol kernel: 3 waves/SIMD since round 6
    cyc_by = {w: sum(COST[w][k] * n[k] for k in CLASSES) for w in set(simds)}
    cyc_s = sum(cyc_by[w] for w in simds) / len(simds)
    cap_s = sum(2 * v / cyc_by[w] for w in simds) / len(simds)
    cap = sum(2 * (v + vy) / (cyc_by[w] + cyc_y) for w in simds) / len(simds)
    checks = {}
    for k, rx in frame_mix.DYN.items():
        d0, d1 = dyn(rx)
        checks[k] = {"model": d0 + u * d1, "measured": meas[k]}
    checks["valu"] = {"model": cls["valu"][0] + u * cls["valu"][1], "measured": v}
    return {
        "waves_per_simd": waves, "items": items, "undecided_fraction": u, "undecided_fraction_simulated": u_sim,
        "undecided_fraction_from_total_valu": u_total, "regen_fraction": g,
        "g_build_instr": len(ins), "g_build_instr_delta": len(ins) - n_plain,
        "item_loop": [hex(item[0]), hex(item[1])], "capture_loops": [[hex(x), hex(y)] for x, y in phil],
        "anchors": a,
        "sync": {"kernel": LONG, "valu_per_item": v, "classes_per_item": {k: n[k] for k in CLASSES},
                 "covered_by_class_counters": covered / v, "uncovered_split": share,
                 "priced_cycles_per_item": cyc_s, "cap_frac": cap_s, "class_check_per_item": checks},
        "sym": {"kernel": SYM, "valu_per_item": vy, "classes_per_item": ny, "priced_cycles_per_item": cyc_y,
                "cap_frac": 2 * vy / cyc_y},
        "cap_frac": cap}


def main(argv):
    dirs = [x for x in argv if not x.startswith("--") and Path(x).is_dir()]
    waves = argv[argv.index("--waves") + 1] if "--waves" in argv else "3,3,3,3"
    summary_p = ROOT / "profiles" / "pmc_summary.json"
    if "--items" in argv:
        items = float(argv[argv.index("--items") + 1])
    else:       # (trial, SNR) items of the profiled command: units / 8 data symbols per frame
        items = json.loads(summary_p.read_text())["frame8"]["units_total_in_run"] / 8
    out = model(dirs, items, waves)
    print(json.dumps({k: out[k] for k in ("cap_frac", "undecided_fraction", "undecided_fraction_simulated",
                                          "undecided_fraction_from_total_valu", "regen_fraction",
                                          "g_build_instr_delta")}, indent=1))
    print(json.dumps({k: out["sync"][k] for k in ("cap_frac", "covered_by_class_counters", "uncovered_split")}))
    print(json.dumps(out["sync"]["class_check_per_item"], indent=1))
    if "--record" in argv:
        ids = json.loads((Path(dirs[0]).parent / "kernel_ids.json").read_text())["ids"]
        out["build_id"] = ids["frame8"]
        (ROOT / "profiles" / "frame8_mix.json").write_text(json.dumps(out, indent=1) + "\n")
        summary = json.loads(summary_p.read_text())
        summary["frame8"]["issue_model"] = {
            "build_id": ids["frame8"], "waves_per_simd": waves, "cap_frac": out["cap_frac"], "method": "classified",
            "undecided_fraction": out["undecided_fraction"], "regen_fraction": out["regen_fraction"],
            "fit": "SQ_INSTS_VALU_FMA_F32; the other class counters measured, the uncovered third split by the assembly",
            "sync_cap_frac": out["sync"]["cap_frac"], "sym_cap_frac": out["sym"]["cap_frac"],
            "source": "tools/frame8_mix.py: every VALU instruction of frame_sync_long_kernel (a -g compile of the same TU "
                      "and flags, instructions attributed to their kernel statements through DWARF inlining records) "
                      "and frame_sym_kernel classified, weighted per item (undecided fraction fitted to SQ_INSTS_VALU "
                      "of %s; regeneration rate tests/golden/frame8_path_rates.json), priced with profiles/r01/ubench/ "
                      "costs; profiles/frame8_mix.json" % ", ".join(str(Path(d).resolve().relative_to(ROOT)) for d in dirs)}
        summary_p.write_text(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
