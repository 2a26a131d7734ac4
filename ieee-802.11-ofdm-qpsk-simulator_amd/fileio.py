"""The reference's file surface (src/OFDM.c:123-143, 1228-1231).

write_float_array_to_file() writes one line of "%.2e" values separated by tabs and ended by a
newline, exactly as OFDM.c does with fprintf on Linux (2-digit exponents, "-inf"), so
scripts/OFDM_Plotting.py and scripts/compare_double.py read the output unchanged.
"""
from __future__ import annotations

import math
import os
from pathlib import Path

import numpy as np

OUTPUT_FILES = ("Output_SNR.txt", "Output_EVM_AGC.txt", "Output_EVM_AGC_DB.txt", "Output_BER.txt")


def _fmt(v: float) -> str:
    # C printf("%.2e") on glibc: inf -> "inf", -inf -> "-inf", nan -> "nan" / "-nan"
    v = float(v)
    if math.isnan(v):
        return "-nan" if math.copysign(1.0, v) < 0 else "nan"
    if math.isinf(v):
        return "inf" if v > 0 else "-inf"
    return "%.2e" % v


def write_float_array_to_file(values, fname: str | os.PathLike) -> None:
    """OFDM.c:123-143 (float values, '%.2e', tab separated, trailing newline)."""
    vals = [float(np.float32(v)) for v in np.asarray(values).ravel()]
    with open(fname, "w") as f:
        f.write("\t".join(_fmt(v) for v in vals))
        f.write("\n")


def write_reference_outputs(out_dir: str | os.PathLike, snr, evm_db, evm_agc_db, ber) -> list[Path]:
    """main()'s four files (OFDM.c:1228-1231): Output_EVM_AGC.txt holds the EVM BEFORE the slicer
    and Output_EVM_AGC_DB.txt the EVM after it (the reference's labels)."""
    d = Path(out_dir)
    if not d.is_dir():
        # OFDM.c:96-100 perror()s and returns when data/ is missing; we refuse loudly instead
        raise FileNotFoundError(f"output directory {d} does not exist")
    paths = [d / n for n in OUTPUT_FILES]
    for p, v in zip(paths, (snr, evm_db, evm_agc_db, ber)):
        write_float_array_to_file(v, p)
    return paths


def write_bits_file(bits, fname: str | os.PathLike) -> None:
    """Code_Output.txt for scripts/compare_double.py: whitespace-separated 0/1 values."""
    with open(fname, "w") as f:
        f.write("\t".join(str(int(b)) for b in np.asarray(bits).ravel()))


def read_float_array_file(fname: str | os.PathLike) -> np.ndarray:
    """Tolerant reader (same token rules as scripts/OFDM_Plotting.py:4-26)."""
    out = []
    for w in Path(fname).read_text().split():
        if "INF" in w or "inf" in w:
            out.append(float("-inf") if "-" in w else float("inf"))
        elif "NaN" in w or "nan" in w or "#J" in w or "#IND" in w:
            out.append(-40.0)
        else:
            out.append(float(w))
    return np.array(out)


def decode_message(bits) -> str:
    """Message_Generator / Binary_To_Decimal (OFDM.c:910-939): 8 bits MSB first per character."""
    b = np.asarray(bits, dtype=np.int64).reshape(-1, 8)
    codes = (b * (1 << np.arange(7, -1, -1))).sum(axis=1)
    return bytes(int(c) & 0xFF for c in codes).decode("latin-1")
