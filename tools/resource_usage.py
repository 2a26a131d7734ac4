"""Per-kernel VGPR / spill / LDS / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python tools/resource_usage.py csrc/ofdm_symbol.hip [extra hipcc flags...]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"


def main(argv):
    src = Path(argv[0])
    if not src.is_absolute():
        src = PKG / src
    sys.path.insert(0, str(PKG))
    from build_lib import CFLAGS, HIPCC, SOURCE_FLAGS
    cmd = [HIPCC, *CFLAGS, *SOURCE_FLAGS.get(src.name, []), *argv[1:], "-c", str(src), "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-4000:])
        return 1
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|"
                      r"Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    dem = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows), capture_output=True, text=True)
    names = dem.stdout.splitlines() if dem.returncode == 0 else [x["name"] for x in rows]
    print(f"{'kernel':70s} {'VGPR':>5s} {'spill':>5s} {'sspill':>6s} {'LDS':>7s} {'occ':>4s}")
    for n, x in zip(names, rows):
        n = re.sub(r"\(.*", "", n).replace("void ", "")
        print(f"{n[:70]:70s} {x.get('VGPRs', '?'):>5s} {x.get('VGPRs Spill', '?'):>5s} {x.get('SGPRs Spill', '?'):>6s} "
              f"{x.get('LDS Size [bytes/block]', '?'):>7s} {x.get('Occupancy [waves/SIMD]', '?'):>4s}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
