"""gcc build of tests/c_caller/ofdm_caller.c against include/ofdm_mi355x.h and libofdm_mi355x.so.

abi_expect.h is generated from the ctypes binding (ofdm_amd.abi.Cfg / RxOpts): the C compiler then asserts
that the header's structs have the offsets and sizes the Python side passes (a mismatch is a compile
error, not a silent misread).  Test infrastructure; __graft_entry__.build() builds the binary in-tree so it
travels to the GPU box with the library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
SRC = HERE / "ofdm_caller.c"
OUT = HERE / "_build"


def abi_expect_header(abi, override: dict | None = None) -> str:
    """X-macro of (struct, field, offset) from the ctypes structs, plus their sizes.  `override` replaces
    entries ({("ofdm_cfg", "kappa"): 16}) so a test can check that a wrong layout fails to compile."""
    override = override or {}
    rows, sizes = [], []
    for cname, st in (("ofdm_cfg", abi.Cfg), ("ofdm_rx_opts", abi.RxOpts)):
        for name, _ in st._fields_:
            off = override.get((cname, name), getattr(st, name).offset)
            rows.append(f"X({cname}, {name}, {off})")
        sizes.append(f"#define ABI_SIZEOF_{cname} {override.get((cname, None), C.sizeof(st))}")
    return ("/* generated from ofdm_amd.abi (ctypes) by tests/c_caller/build_caller.py */\n"
            "#define ABI_FIELDS(X) " + " ".join(rows) + "\n" + "\n".join(sizes) + "\n")


def build(abi, lib: Path, out_dir: Path = OUT, override: dict | None = None) -> Path:
    """Compile + link the caller (rpath to the library's directory).  Raises RuntimeError with gcc's
    output on failure."""
    out_dir.mkdir(parents=True, exist_ok=True)
    (out_dir / "abi_expect.h").write_text(abi_expect_header(abi, override))
    exe = out_dir / "ofdm_caller"
    lib = Path(lib).resolve()
    # rpath relative to the executable: the tree moves (the GPU box runs a copy of it)
    rpath = "$ORIGIN/" + os.path.relpath(lib.parent, out_dir.resolve())
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT / 'include'}", f"-I{out_dir}",
           str(SRC), "-o", str(exe), f"-L{lib.parent}", "-l:" + lib.name, f"-Wl,-rpath,{rpath}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed:\n{r.stderr[-4000:]}")
    return exe
