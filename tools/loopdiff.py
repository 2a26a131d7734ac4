"""Compare one loop body of a kernel in two gfx950 assembly files, modulo register names.

usage: python tools/loopdiff.py A.s B.s <mangled kernel> LOOP_A LOOP_B
(LOOP_x: the loop's rank by size, as tools/isa_mix.py --loop picks it; the SNR loop of the packed receivers
is the one whose VALU count isa_mix reports as the issue model's loop_valu.)

Prints the instruction counts and how many lines differ (a) in any way, (b) beyond SGPR names, (c) beyond
all register names.  K3c's SNR-loop schedule moves with unrelated prologue code (profiles/r03/ab_h): a kernel
A/B is only read as a change of the code it edits when (c) is 0.
"""
import difflib
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from isa_mix import loop_body  # noqa: E402

SGPR = re.compile(r"\bs\[?\d+(:\d+\])?")
VGPR = re.compile(r"\bv\[?\d+(:\d+\])?")


def loop_lines(path, name, which):
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
    body = text[start:end]
    a, b = loop_body(body, which)
    out = []
    for l in body[a:b]:
        l = l.split(";")[0].strip()
        if l:
            out.append(re.sub(r"\.LBB\d+_\d+", "L", l))
    return out


def ndiff(x, y):
    return sum(1 for d in difflib.unified_diff(x, y, lineterm="", n=0)
               if d[:1] in "+-" and not d.startswith(("+++", "---")))


def main(argv):
    pa, pb, name, la, lb = argv[0], argv[1], argv[2], int(argv[3]), int(argv[4])
    x, y = loop_lines(pa, name, la), loop_lines(pb, name, lb)
    nos = lambda v: [SGPR.sub("S", l) for l in v]                     # noqa: E731
    noreg = lambda v: [VGPR.sub("V", l) for l in nos(v)]             # noqa: E731
    print(f"lines {len(x)} / {len(y)}; differing: any {ndiff(x, y)}, beyond SGPR names {ndiff(nos(x), nos(y))}, "
          f"beyond register names {ndiff(noreg(x), noreg(y))}")


if __name__ == "__main__":
    main(sys.argv[1:])
