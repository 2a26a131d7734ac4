"""Build libofdm_mi355x.so in-tree with hipcc for gfx950 (MI355X).

The HIP translation units in csrc/ are compiled in parallel and linked into one shared library
next to this file, so the .so travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
INCLUDE = PKG_DIR.parent / "include"
BUILD = PKG_DIR / "_build"
LIB = PKG_DIR / "libofdm_mi355x.so"
SOURCES = ["ofdm_capi.hip", "ofdm_symbol.hip", "ofdm_rxpack.hip", "ofdm_rxpack_ideal.hip", "ofdm_frame.hip",
           "ofdm_frame_sym.hip", "ofdm_frame_fix.hip", "ofdm_frame_long.hip"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-slp-vectorize: keep f32 math scalar (packed v_pk_* f32 gives no rate on gfx950 and its
#   register-pair shuffles cost VGPRs); -fno-signed-zeros lets x+0 fold in the sparse Tx IFFT;
#   no atomic optimizer: counter atomics are already wave-reduced.
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "-fno-signed-zeros",
          "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", f"-I{INCLUDE}", f"-I{CSRC}"]


# per-source flags: the symbol-mode kernels schedule for ILP (A/B: c3 +1 %, c2 +3 %, c5 +3 %; the
# frame kernels -0.5 %, profiles/r01/ab/ab_*_ilp.json; packed receivers c3 +1.4 %, c2 +2.5 %,
# profiles/r02/ab/SUMMARY.md).  The packed ideal-CSI receivers (ofdm_rxpack_ideal.hip) keep the default scheduler:
# with the prologue's Tx builds, max-ILP spills them at their 168-VGPR budget.  The fixed-geometry frame sync kernel
# (ofdm_frame_fix.hip) schedules iterative-ILP and the long-capture kernel (ofdm_frame_long.hip) max-ILP (round 6,
# interleaved: frame +0.9 % over max-ILP; frame8 +0.8 % over the default -- iterative-ILP +0.7 %, but the compiler
# fails on that TU with -g, which tools/frame8_mix.py needs; the symbol kernel's TU is best at the default,
# profiles/r06/frame/ab_sched.txt).
SOURCE_FLAGS = {"ofdm_symbol.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                "ofdm_rxpack.hip": os.environ.get("OFDM_RXPACK_FLAGS", "-mllvm -amdgpu-sched-strategy=max-ilp").split(),
                "ofdm_rxpack_ideal.hip": os.environ.get("OFDM_RXPACK_IDEAL_FLAGS", "").split(),
                "ofdm_frame.hip": os.environ.get("OFDM_FRAME_FLAGS", "").split(),
                "ofdm_frame_sym.hip": os.environ.get("OFDM_FRAME_SYM_FLAGS", "").split(),
                "ofdm_frame_fix.hip": os.environ.get("OFDM_FRAME_FIX_FLAGS",
                                                     "-mllvm -amdgpu-sched-strategy=iterative-ilp").split(),
                "ofdm_frame_long.hip": os.environ.get("OFDM_FRAME_LONG_FLAGS",
                                                      "-mllvm -amdgpu-sched-strategy=max-ilp").split()}


# Kernels whose parity-dump variants (last template argument `true`) are allowed to spill: they
# write every equalised bin and run only in tests.  Every other kernel must build spill-free.
DUMP_KERNEL = re.compile(r"^ofdm::(rx_\w+_kernel<.*true>|frame_sym_kernel<true, \d+>)$")
RESOURCE_REPORT = BUILD / "resource_usage.json"


def parse_resource_usage(stderr: str) -> list[dict]:
    """Per-kernel rows of hipcc's -Rpass-analysis=kernel-resource-usage remarks (demangled names)."""
    rows, cur = [], None
    for line in stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs|SGPRs Spill|ScratchSize \[bytes/lane\]|"
                      r"LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"mangled": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = int(v) if v.lstrip("-").isdigit() else v
    dem = subprocess.run(["c++filt"], input="\n".join(x["mangled"] for x in rows), capture_output=True, text=True)
    names = dem.stdout.splitlines() if dem.returncode == 0 and rows else [x["mangled"] for x in rows]
    for x, n in zip(rows, names):
        x["name"] = re.sub(r"\(.*", "", n).replace("void ", "")
        x["dump_variant"] = bool(DUMP_KERNEL.match(x["name"]))
    return rows


def spilling_kernels(rows: list[dict]) -> list[str]:
    """Non-dump kernels with a VGPR spill or scratch use (SGPR spills land in VGPR lanes, not scratch)."""
    return [f"{x['name']}: {x.get('VGPRs Spill')} VGPR spilled, {x.get('ScratchSize [bytes/lane]')} B scratch/lane"
            for x in rows if not x["dump_variant"]
            and (x.get("VGPRs Spill", 0) or x.get("ScratchSize [bytes/lane]", 0))]


def _compile(src: str, extra: list[str], build_dir: Path = BUILD) -> tuple[Path, list[dict]]:
    obj = build_dir / (Path(src).stem + ".o")
    cmd = [HIPCC, *CFLAGS, *SOURCE_FLAGS.get(src, []), *extra, "-c", str(CSRC / src), "-o", str(obj),
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    rows = parse_resource_usage(r.stderr)
    for x in rows:
        x["source"] = src
    return obj, rows


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = list(CSRC.glob("*")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, extra: list[str] | None = None, verbose: bool = True,
          out: Path | None = None) -> Path:
    """Build the library (default: in-tree LIB).  `out` + `extra` make a variant build (own objects)."""
    lib = Path(out) if out else LIB
    if out is None and not force and not _stale():
        return LIB
    build_dir = BUILD if out is None else lib.parent / ("_build_" + lib.stem)
    build_dir.mkdir(parents=True, exist_ok=True)
    extra = extra or []
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        done = list(ex.map(lambda s: _compile(s, extra, build_dir), SOURCES))
    objs = [o for o, _ in done]
    rows = [x for _, r in done for x in r]
    (build_dir / RESOURCE_REPORT.name).write_text(json.dumps(rows, indent=1))
    if out is None:
        bad = spilling_kernels(rows)
        if bad:
            raise RuntimeError("kernels on the product path spill to scratch:\n  " + "\n  ".join(bad))
    tmp = lib.with_suffix(".so.tmp")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, lib)
    if verbose:
        print(f"built {lib}", file=sys.stderr)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
