"""Import helper for the product package, whose directory name
(`ieee-802.11-ofdm-qpsk-simulator_amd/`) is not a Python identifier.  load() registers it as the
module `ofdm_amd`; build() compiles libofdm_mi355x.so for gfx950 in-tree."""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd"
PKG_NAME = "ofdm_amd"


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(PKG_NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod


def build(force: bool = False):
    load()
    from ofdm_amd import build_lib  # noqa: PLC0415
    return build_lib.build(force=force)


if __name__ == "__main__":
    # python ofdm_pkg.py build [--force]      compile libofdm_mi355x.so
    # python ofdm_pkg.py sweep [args...]      OFDM.c main() on the GPU (see ofdm_amd.sweep)
    cmd = sys.argv[1] if len(sys.argv) > 1 else "build"
    if cmd == "sweep":
        load()
        from ofdm_amd import sweep  # noqa: PLC0415
        sweep.main(sys.argv[2:])
    else:
        print(build(force="--force" in sys.argv))
