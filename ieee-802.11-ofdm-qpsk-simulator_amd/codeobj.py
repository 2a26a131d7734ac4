"""Kernel build ids read from the shipped library's gfx950 code objects.

A PMC record (profiles/pmc_summary.json) is a measurement of ONE build of a kernel: its VALU instruction
count per unit is only valid for that machine code.  `kernel_build_id` hashes a kernel's code bytes and its
kernel descriptor (VGPR/SGPR/LDS/scratch settings) straight from the .so, so the profiling run can stamp its
record and bench.py can refuse a record whose id differs from the library it actually loaded.

Pure Python (struct + hashlib) on the ELF layout: the .so's .hip_fatbin section holds one clang offload bundle
per translation unit ("__CLANG_OFFLOAD_BUNDLE__", entry table of (offset, size, triple)); the gfx950 entry is
an AMDGPU ELF64 code object whose .symtab names each kernel (STT_FUNC, its code) and `<kernel>.kd`
(STT_OBJECT, its 64-byte descriptor).
"""
from __future__ import annotations

import hashlib
import re
import struct
from functools import lru_cache
from pathlib import Path

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "gfx950"

# the kernels a workload's PMC record measures, as mangled-name fragments of their instantiations
# (template arguments <KIND, CONV, CHAN, DUMP>; ofdm_rxpack.hip launch_rx_pack, ofdm_frame.hip)
WORKLOAD_KERNELS = {
    "c3": ("rx_pack_kernelILi2ELi0ELi0ELb0E",),
    "c4": ("rx_pack_kernelILi2ELi0ELi0ELb0E",),
    "c5": ("rx_pack_kernelILi2ELi0ELi1ELb0E",),
    "c2": ("rx_pack_kernelILi0ELi0ELi0ELb0E",),
    "frame": ("frame_sync_kernelILi2ELi3008E", "frame_sym_kernelILb0ELi2E"),
    # frame8: the long-capture sync kernel (ofdm_frame_long.hip; run_frame_chunk picks it for captures > 4,100
    # samples) and the generic symbol kernel
    "frame8": ("frame_sync_long_kernel", "frame_sym_kernelILb0ELi0E"),
    "fft64": ("fft64_lds_kernelILb0ELi0E", "fft64_lds_kernelILb1ELi0E"),
}


def _bundles(blob: bytes):
    """(triple, bytes) of every offload-bundle entry in the file."""
    pos = blob.find(BUNDLE_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        o = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, o)
            triple = blob[o + 24:o + 24 + tlen].decode()
            o += 24 + tlen
            yield triple, blob[pos + off:pos + off + size]
        pos = blob.find(BUNDLE_MAGIC, o)


def _elf_symbols(elf: bytes, with_type: bool = False):
    """{name: bytes} (with_type: {name: (STT type, bytes)}) of every sized FUNC / OBJECT symbol of an ELF64
    little-endian code object."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return {}
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for s in secs:
        if s[1] != 2:                      # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for i in range(s[5] // s[9]):
            name_off, info, _, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s[4] + i * s[9])
            if size == 0 or shndx == 0 or shndx >= len(secs) or (info & 0xF) not in (1, 2):
                continue
            so = strtab[4] + name_off
            name = elf[so:elf.index(b"\0", so)].decode()
            sec = secs[shndx]                # sh_addr, sh_offset: file offset of the symbol's bytes
            start = sec[4] + (value - sec[3])
            out[name] = (info & 0xF, elf[start:start + size]) if with_type else elf[start:start + size]
    return out


@lru_cache(maxsize=8)
def _code_objects(path: str, mtime: float) -> list:
    """[{name: (STT type, bytes)}] per gfx950 code object (one per translation unit)"""
    blob = Path(path).read_bytes()
    return [_elf_symbols(body, with_type=True) for triple, body in _bundles(blob) if triple.endswith(TARGET)]


def _symbols(path: str, mtime: float) -> dict:
    return {n: b for co in _code_objects(path, mtime) for n, (_, b) in co.items()}


def kernel_symbols(lib_path) -> dict:
    """{mangled name: code or descriptor bytes} of the gfx950 code objects inside the library."""
    p = Path(lib_path)
    return _symbols(str(p), p.stat().st_mtime)


STT_FUNC = 2


def kernel_build_id(lib_path, fragments) -> str | None:
    """sha256 (first 16 hex digits) over the code and kernel descriptor (its code-entry offset zeroed) of every
    kernel whose mangled name contains one of `fragments`, and over every non-kernel function of the code objects
    holding them (a device function the compiler did not inline is code the kernel runs: ADVICE r3); None when no
    kernel matches.  The kernels' constant data is their descriptors (.rodata holds nothing else here)."""
    p = Path(lib_path)
    h = hashlib.sha256()
    found = False
    for co in _code_objects(str(p), p.stat().st_mtime):
        names = sorted(n for n in co if any(re.search(re.escape(f), n) for f in fragments))
        if not names:
            continue
        found = True
        callees = sorted(n for n, (t, _) in co.items()
                         if t == STT_FUNC and not n.endswith(".kd") and n + ".kd" not in co)
        for n in names + callees:
            h.update(n.encode() + b"\0" + _layout_free(n, co[n][1]))
    return h.hexdigest()[:16] if found else None


def _layout_free(name: str, body: bytes) -> bytes:
    """A kernel descriptor's kernel_code_entry_byte_offset (bytes 16-23: descriptor to code entry) depends on
    where the linker placed the code, which moves when any other kernel of the library changes size; it is
    zeroed, so that the id changes with the kernel's own code and descriptor only."""
    if name.endswith(".kd") and len(body) == 64:
        return body[:16] + bytes(8) + body[24:]
    return body


def workload_build_id(lib_path, workload: str) -> str | None:
    frags = WORKLOAD_KERNELS.get(workload)
    return kernel_build_id(lib_path, frags) if frags else None
