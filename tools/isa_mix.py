"""Issue-cost model of a kernel's SNR-loop body from its gfx950 assembly.

usage: python tools/isa_mix.py <asm.s> <mangled kernel name> [--loop N]

Classes follow the measured issue costs (profiles/r01/ubench/ubench_bank_forms.txt, SIMD cycles per
wave64 instruction at 2 / 4 waves per SIMD):
  fast   v_add/sub/mul/fma/fmac/fmamk/fmaak_f32, v_add/sub_u32, v_and/or/xor_b32, v_bitop3_b32 with
         VGPR / inline-constant operands (and VOP2 literals); v_bitop3_b32 also with an SGPR operand
         (measured in the receivers, profiles/r03/ab_o)                          2.35 / 1.97
  slow   any SGPR operand; shifts, alignbit, cvt, max/min, bfe, perm, mul_lo/hi, DPP, cndmask_e64,
         v_mad_u64_u32 (3.22 at 4 waves)                                         4.30 / 3.15
  trans  v_log/sin/cos/sqrt/rcp/exp_f32                                          8.23 / 6.12
  cnd    v_cndmask_b32_e32 (VCC)                                                 16.2 / 12.5
The loop is the largest basic block between a label and its backward branch (or --loop N: the N-th
largest)."""
import collections
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

FAST_OPS = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|fmamk|fmaak)_f32|^v_(add|sub|subrev)_u32|^v_(and|or|xor)_b32"
                      r"|^v_bitop3_b32|^v_mov_b32|^v_add_co_u32|^v_sub_co_u32")
TRANS = re.compile(r"^v_(log|sin|cos|sqrt|rcp|exp|rsq)_f32")
# v_bitop3_b32 with an SGPR operand (the Philox round keys) issues at the fast rate inside the receivers: moving
# the keys to VGPRs measured +0.3 % (20 VGPRs of keys) and -4 % (2 VGPRs advanced per round, +240 v_add per
# iteration) on c3, where the SGPR-slow pricing predicted +5 % (profiles/r03/ab_o/), unlike the isolated
# microbenchmark form of profiles/r01/ubench
SGPR_FAST = re.compile(r"^v_bitop3_b32")
COST = {2: {"fast": 2.35, "slow": 4.30, "trans": 8.23, "cnd": 16.2},
        4: {"fast": 1.97, "slow": 3.15, "trans": 6.12, "cnd": 12.5}}
COST[3] = {k: 0.5 * (COST[2][k] + COST[4][k]) for k in COST[2]}     # interpolated (not measured)


def classify(op, args):
    if op.startswith(("s_", "ds_", "global_", "buffer_", "scratch_", "flat_")):
        return op.split("_")[0]
    if not op.startswith("v_"):
        return None
    if TRANS.match(op):
        return "trans"
    if op.startswith("v_cndmask_b32_e32") or (op.startswith("v_cndmask") and "vcc" in args):
        return "cnd"
    sgpr = re.search(r"(?<![\w])s\d+|s\[\d+", args) is not None
    if "dpp" in args or "quad_perm" in args or "row_" in args:
        return "slow"
    if FAST_OPS.match(op) and (not sgpr or SGPR_FAST.match(op)):
        return "fast"
    return "slow"


def loop_body(lines, which=1):
    """(start, end) line ranges of basic blocks ending with a backward branch to their label"""
    labels = {}
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            out.append((i - labels[m.group(1)], labels[m.group(1)], i))
    out.sort(reverse=True)
    return out[which - 1][1:]


def main(argv):
    path, name = argv[0], argv[1]
    which = int(argv[argv.index("--loop") + 1]) if "--loop" in argv else 1
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
    body = text[start:end]
    a, b = loop_body(body, which)
    cls = collections.Counter()
    ops = collections.Counter()
    for l in body[a:b]:
        t = l.strip().split(None, 1)
        if not t or t[0].startswith((";", ".")):
            continue
        op, args = t[0], (t[1] if len(t) > 1 else "")
        c = classify(op, args)
        if c:
            cls[c] += 1
            ops[(c, op)] += 1
    valu = sum(cls[k] for k in ("fast", "slow", "trans", "cnd"))
    print(f"loop lines {a}-{b}: VALU {valu}  " + "  ".join(f"{k} {v}" for k, v in sorted(cls.items())))
    priced = {}
    for w in (2, 3, 4):
        cyc = sum(COST[w][k] * cls[k] for k in COST[w])
        priced[w] = cyc
        # the nominal issue peak is one wave-instruction per 2 SIMD cycles: this mix can reach 2 VALU / cyc of it
        print(f"  priced issue cycles at {w} waves/SIMD: {cyc:.0f}  (mix cap: {2 * valu / cyc:.3f} of the nominal peak)")
    for (c, op), n in ops.most_common(40):
        print(f"  {c:6s} {op:28s} {n}")
    if "--record" in argv:       # --record WORKLOAD --waves W: store the cap beside the workload's PMC summary
        wl = argv[argv.index("--record") + 1]
        w = int(argv[argv.index("--waves") + 1]) if "--waves" in argv else 2
        out = ROOT / "profiles" / "pmc_summary.json"
        summary = json.loads(out.read_text())
        sys.path.insert(0, str(ROOT / "tools"))
        from kernel_ids import ids  # noqa: PLC0415
        summary[wl]["issue_model"] = {
            # the assembly is compiled from the same sources and flags as the in-tree library: its build id
            "build_id": ids()["ids"].get(wl),
            "kernel": name, "loop_valu": valu, "classes": dict(cls), "waves_per_simd": w,
            "priced_cycles": priced[w], "cap_frac": 2 * valu / priced[w],
            "source": "tools/isa_mix.py on the gfx950 assembly; class costs profiles/r01/ubench/"}
        out.write_text(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
