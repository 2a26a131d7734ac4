"""Per-kernel VGPR / spill / LDS / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python tools/resource_usage.py [csrc/ofdm_symbol.hip [extra hipcc flags...]]
With no source: print the report the last in-tree build wrote (_build/resource_usage.json).
"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"
sys.path.insert(0, str(PKG))
import build_lib  # noqa: E402


def table(rows):
    print(f"{'kernel':70s} {'VGPR':>5s} {'spill':>5s} {'sspill':>6s} {'LDS':>7s} {'occ':>4s}")
    for x in rows:
        print(f"{x['name'][:70]:70s} {x.get('VGPRs', '?')!s:>5s} {x.get('VGPRs Spill', '?')!s:>5s} "
              f"{x.get('SGPRs Spill', '?')!s:>6s} {x.get('LDS Size [bytes/block]', '?')!s:>7s} "
              f"{x.get('Occupancy [waves/SIMD]', '?')!s:>4s}")


def main(argv):
    if not argv:
        table(json.loads(build_lib.RESOURCE_REPORT.read_text()))
        return 0
    src = Path(argv[0])
    if not src.is_absolute():
        src = PKG / src
    cmd = [build_lib.HIPCC, *build_lib.CFLAGS, *build_lib.SOURCE_FLAGS.get(src.name, []), *argv[1:], "-c",
           str(src), "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-4000:])
        return 1
    table(build_lib.parse_resource_usage(r.stderr))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
