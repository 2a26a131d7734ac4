"""Build compile-flag variants of the library under variants/ for A/B timing on the GPU box.

usage: python tools/build_variants.py NAME=-DFLAG[,-DFLAG2] ...
then on the box: OFDM_MI355X_LIB=variants/libofdm_NAME.so python bench.py ...
"""
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"))
import build_lib  # noqa: E402


def main(argv):
    specs = [a.split("=", 1) for a in argv]
    out = ROOT / "variants"
    out.mkdir(exist_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, len(specs))) as ex:
        list(ex.map(lambda s: build_lib.build(extra=[f for f in s[1].split(",") if f],
                                              out=out / f"libofdm_{s[0]}.so"), specs))


if __name__ == "__main__":
    main(sys.argv[1:])
