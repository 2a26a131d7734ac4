"""Per-basic-block instruction counts of one kernel in a gfx950 .s file (loop depth from LLVM's
comments), to see which blocks of a kernel carry its VALU / SALU / LDS work.

usage: python tools/bb_mix.py <asm.s> <kernel-name substring> [min VALU per block]
"""
import re
import sys


def main(path, kname, min_v=6):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\w*{kname}\w*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    cur = {"name": "entry", "line": start + 1, "depth": 0, "v": 0, "s": 0, "ds": 0, "g": 0, "t": 0, "f64": 0, "cnd": 0}
    out = [cur]
    for i in range(start + 1, end + 1):
        l = lines[i].strip()
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):(.*)", l)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2) + (lines[i + 1] if i + 1 < len(lines) else ""))
            cur = {"name": m.group(1), "line": i + 1, "depth": int(d.group(1)) if d else 0,
                   "v": 0, "s": 0, "ds": 0, "g": 0, "t": 0, "f64": 0, "cnd": 0}
            out.append(cur)
            continue
        if not l or l[0] in ";.":
            continue
        op = l.split()[0]
        if op.startswith("v_"):
            cur["v"] += 1
            cur["t"] += bool(re.match(r"v_(sin|cos|log|exp|sqrt|rcp|rsq)_", op))
            cur["f64"] += "f64" in op
            cur["cnd"] += op.startswith("v_cndmask")
        elif op.startswith("s_"):
            cur["s"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("global_", "buffer_")):
            cur["g"] += 1
    print(f"{'block':12s} {'line':>6s} {'dep':>3s} {'VALU':>5s} {'SALU':>5s} {'LDS':>4s} {'GMEM':>4s} {'trans':>5s} {'f64':>4s} {'cnd':>4s}")
    for c in out:
        if c["v"] >= min_v or c["ds"] >= 4:
            print(f"{c['name']:12s} {c['line']:6d} {c['depth']:3d} {c['v']:5d} {c['s']:5d} {c['ds']:4d} {c['g']:4d} "
                  f"{c['t']:5d} {c['f64']:4d} {c['cnd']:4d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 6)
