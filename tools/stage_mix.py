"""Per-stage instruction budget of the c3 receiver's SNR loop (rx_pack_kernel<2, C, AWGN>), VERDICT r4 item 4.

usage: python tools/stage_mix.py [--record profiles/r05/c3_stages.json] [--kernel c3|c5]

The SNR loop is compiled (device-only gfx950 assembly, the library's own flags) once as built and once per stage
ablation (ofdm_rxpack.hip OFDM_ABL_*); a stage's instructions are the loop's VALU count minus the ablated build's,
plus what the ablation leaves in its place (counted below from the replacement code), classified and priced as in
tools/isa_mix.py (SIMD cycles per wave-instruction at 2 waves/SIMD).  Whatever no ablation removes (LDS address
arithmetic, the Hermitian pair untangling of the data noise, loop control) is the remainder row.

The OFDM_ABL_* ablations were pruned from csrc/ in round 6 (profiles/r06/README.md): run this tool in a checkout of
commit aec0f2e (`git worktree add /tmp/abl aec0f2e`).

Per frame and SNR point the loop draws 48 Philox blocks (16 for the LTF pair, 32 for the data windows) and 96 Box-
Muller pairs, runs one 32-point (LTF pair) and one 64-point complex (D0 + j D1) FFT, 24 bin pairs of estimate /
equaliser / slicer / demap for both data symbols, and one frame's counters.
"""
from __future__ import annotations

import collections
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import build_lib  # noqa: E402
import isa_mix  # noqa: E402

KERNELS = {"c3": "_ZN4ofdm14rx_pack_kernelILi2ELi0ELi0ELb0EEEvNS_6RxArgsE",
           "c5": "_ZN4ofdm14rx_pack_kernelILi2ELi0ELi1ELb0EEEvNS_6RxArgsE"}
# stage -> (ablation macro, VALU the ablation leaves per loop iteration in the stage's place, by class)
#   NO_PHILOX: per block one v_xor + v_mad_u64_u32 + two v_xor (48 blocks)
#   NO_BM:     per block 4 cvt + 4 mul (48 blocks)
#   the others leave nothing of their own (NO_EQ: 5 adds per pair, 24 pairs)
STAGES = [("Philox4x32-10 (48 blocks)", "OFDM_ABL_NO_PHILOX", {"fast": 48 * 3, "slow": 48 * 1}),
          ("Box-Muller (96 pairs)", "OFDM_ABL_NO_BM", {"slow": 48 * 4, "fast": 48 * 4}),
          ("data FFT (64-point complex, D0 + j D1)", "OFDM_ABL_NO_DFFT", {}),
          ("LTF-pair FFT (32-point)", "OFDM_ABL_NO_LFFT", {}),
          ("estimate + equaliser + slicer + demap (24 pairs x 2 symbols)", "OFDM_ABL_NO_EQ", {"fast": 24 * 6}),
          ("frame counters (metrics + LDS flush)", "OFDM_ABL_NO_CNT", {})]
CLASSES = ("fast", "slow", "trans", "cnd")


def loop_mix(flags: list[str], kernel: str) -> collections.Counter:
    src = build_lib.CSRC / "ofdm_rxpack.hip"
    cmd = [build_lib.HIPCC, *build_lib.CFLAGS, *build_lib.SOURCE_FLAGS["ofdm_rxpack.hip"], *flags,
           "--cuda-device-only", "-S", str(src), "-o", "-"]
    asm = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout.splitlines()
    start = next(i for i, l in enumerate(asm) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(asm)) if "s_endpgm" in asm[i])
    body = asm[start:end]
    # the SNR loop: the largest backward loop that is (nearly) free of scalar instructions -- the item loops that
    # enclose it carry the prologue's scalar address and control work (> 9 % of their VALU count; the SNR loop 1 %)
    best = None
    for k in range(1, 64):
        try:
            a, b = isa_mix.loop_body(body, k)
        except IndexError:
            break
        cls = collections.Counter()
        for l in body[a:b]:
            t = l.strip().split(None, 1)
            if not t or t[0].startswith((";", ".")):
                continue
            c = isa_mix.classify(t[0], t[1] if len(t) > 1 else "")
            if c:
                cls[c] += 1
        v = sum(cls[x] for x in CLASSES)
        if v > 1000 and cls["s"] <= 0.03 * v and (best is None or v > sum(best[x] for x in CLASSES)):
            best = cls
    return best


def priced(cls) -> float:
    return sum(isa_mix.COST[2][k] * cls.get(k, 0) for k in CLASSES)


def main(argv):
    which = argv[argv.index("--kernel") + 1] if "--kernel" in argv else "c3"
    kernel = KERNELS[which]
    full = loop_mix([], kernel)
    rows = []
    total_v = sum(full[k] for k in CLASSES)
    total_c = priced(full)
    acc = collections.Counter()
    for name, macro, left in STAGES:
        ab = loop_mix([f"-D{macro}"], kernel)
        st = collections.Counter({k: full[k] - ab[k] + left.get(k, 0) for k in CLASSES})
        acc.update(st)
        rows.append((name, macro, st))
    rest = collections.Counter({k: full[k] - acc[k] for k in CLASSES})
    rows.append(("remainder (addresses, noise untangling, LDS operand staging, loop control)", "-", rest))
    print(f"{which} SNR loop: {total_v} VALU, {total_c:.0f} priced SIMD cycles at 2 waves/SIMD "
          f"(mix cap {2 * total_v / total_c:.3f} of nominal)")
    print(f"{'stage':66s} {'VALU':>6s} {'%':>6s} {'cycles':>7s} {'%':>6s}  fast slow trans cnd")
    out = []
    for name, macro, st in rows:
        v = sum(st[k] for k in CLASSES)
        c = priced(st)
        print(f"{name:66s} {v:6d} {100 * v / total_v:5.1f}% {c:7.0f} {100 * c / total_c:5.1f}%  "
              + " ".join(f"{st[k]:4d}" for k in CLASSES))
        out.append({"stage": name, "ablation": macro, "valu": v, "valu_share": v / total_v, "priced_cycles": c,
                    "cycle_share": c / total_c, "classes": dict(st)})
    if "--record" in argv:
        p = Path(argv[argv.index("--record") + 1])
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps({"kernel": kernel, "loop_valu": total_v, "loop_priced_cycles": total_c,
                                 "waves_per_simd": 2, "class_costs": isa_mix.COST[2], "stages": out,
                                 "source": "tools/stage_mix.py: ablation deltas of the gfx950 assembly"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
