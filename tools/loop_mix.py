"""Instruction mix of the largest basic block (the SNR-loop body) of a kernel.

usage: python tools/loop_mix.py <mangled-kernel-substring> [csrc/file.hip]
"""
import collections
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"
sys.path.insert(0, str(PKG))
from build_lib import CFLAGS, HIPCC, SOURCE_FLAGS  # noqa: E402

# issue cost (SIMD cycles per wave-instruction, 2 waves/SIMD) measured by tools/ubench_valu.hip
COST2 = {"transc": 8.34, "mad64": 5.02, "dpp": 4.45, "3src": 4.33, "2src": 2.73}
TRANSC = ("v_log_f32", "v_sin_f32", "v_cos_f32", "v_sqrt_f32", "v_rcp_f32", "v_exp_f32", "v_rsq_f32")
THREE = ("v_fma", "v_fmac", "v_bitop3", "v_cndmask", "v_add3", "v_lshl_add", "v_fmamk", "v_fmaak", "v_or3",
         "v_alignbit", "v_bfi", "v_lshl_or", "v_and_or", "v_perm", "v_med3", "v_max3", "v_min3", "v_mad_u32",
         "v_bfe")


def cat(op):
    if "dpp" in op:
        return "dpp"
    if op.startswith(TRANSC):
        return "transc"
    if op.startswith("v_mad_u64"):
        return "mad64"
    if op.startswith(THREE):
        return "3src"
    return "2src"


def main(argv):
    pat = argv[0]
    src = PKG / (argv[1] if len(argv) > 1 else "csrc/ofdm_symbol.hip")
    s = subprocess.run([HIPCC, *CFLAGS, *SOURCE_FLAGS.get(src.name, []), "--cuda-device-only", "-S", str(src), "-o", "-"], capture_output=True,
                       text=True, check=True).stdout
    names = [m.group(1) for m in re.finditer(r"^(_Z\S*):", s, re.M) if pat in m.group(1)]
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        blocks, cur = [], None
        for line in s[i:j].splitlines():
            if re.match(r"^\.LBB\d+_\d+:", line):
                cur = collections.Counter()
                blocks.append(cur)
                continue
            t = line.strip()
            if cur is not None and t and not t.startswith((".", ";")):
                cur[t.split()[0]] += 1
        big = max(blocks, key=lambda b: sum(b.values()))
        valu = {k: v for k, v in big.items() if k.startswith("v_")}
        cats = collections.Counter()
        for k, v in valu.items():
            cats[cat(k)] += v
        cyc = sum(COST2[c] * n for c, n in cats.items())
        print(f"{name}: VALU {sum(valu.values())}  est {cyc:.0f} SIMD cycles @2 waves/SIMD  "
              + "  ".join(f"{c}={n}" for c, n in cats.most_common())
              + f"  ds={sum(v for k, v in big.items() if k.startswith('ds_'))}"
              + f"  salu={sum(v for k, v in big.items() if k.startswith('s_'))}")
        if "-v" in argv:
            for k, v in big.most_common(40):
                print(f"   {k:28s}{v}")


if __name__ == "__main__":
    main(sys.argv[1:])
