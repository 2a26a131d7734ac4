"""Build the device test programs (tests/test_gpu_device.py) in-tree with the library's own hipcc flags, so that
the inlined device functions they exercise compile as they do inside the kernels.  Called by
__graft_entry__.build(); the binaries travel to the GPU box with the snapshot."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
OUT = HERE / "_build"
PROGRAMS = ["atan2_check"]


def build() -> list[Path]:
    root = HERE.parents[1]
    sys.path.insert(0, str(root))
    import ofdm_pkg
    ofdm_pkg.load()
    from ofdm_amd import build_lib as bl  # noqa: PLC0415
    OUT.mkdir(exist_ok=True)
    out = []
    for p in PROGRAMS:
        exe = OUT / p
        src = HERE / f"{p}.hip"
        if not exe.exists() or exe.stat().st_mtime < max(src.stat().st_mtime, (bl.CSRC / "ofdm_device.h").stat().st_mtime):
            flags = [f for f in bl.CFLAGS if f != "-fPIC"]
            r = subprocess.run([bl.HIPCC, *flags, str(src), "-o", str(exe)], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
        out.append(exe)
    return out


if __name__ == "__main__":
    print(build())
