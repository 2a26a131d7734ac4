"""ctypes binding of the C ABI in include/ofdm_mi355x.h (libofdm_mi355x.so).

The library is the product: there is no CPU or PyTorch fallback.  If the shared object is
missing or cannot be loaded, load_library() raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libofdm_mi355x.so"
HEADER = PKG_DIR.parent / "include" / "ofdm_mi355x.h"

ABI_VERSION = 1

# enums (include/ofdm_mi355x.h)
CONV = {"c": 0, "matlab": 1}
PAYLOAD = {"random": 0, "message": 1, "tester": 2}
EST = {"ls": 0, "ideal": 1}
NOISE = {"real": 0, "complex": 1, "none": 2}
CHANNEL = {"awgn": 0, "rayleigh4": 1}

# counters
NCOUNTERS = 16
C_FRAMES, C_SYMBOLS, C_BITS, C_BIT_ERR, C_FRAME_ERR, C_SYNC_FAIL, C_EVM_TERMS, C_EVM_PRE_Q, \
    C_EVM_POST_AXIS, C_EVMDB_PRE_Q, C_EVMDB_POST_Q, C_EVMDB_POST_FINITE, C_OOB, \
    C_WL_MIN_Q, C_WL_MAX_Q, C_WL_BITS = range(16)
EVM_Q_SCALE = float(1 << 20)

# kernel ids for timing
K_FFT, K_TX, K_RX, K_FRAME = range(4)

# every entry point of the header, with ctypes argument types
_V = C.c_void_p
_SIGS = {
    "ofdm_abi_version": (C.c_int, []),
    "ofdm_last_error": (C.c_char_p, []),
    "ofdm_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "ofdm_ctx_create": (C.c_int, [C.c_int, C.POINTER(_V)]),
    "ofdm_ctx_destroy": (C.c_int, [_V]),
    "ofdm_ctx_set_stream": (C.c_int, [_V, _V]),
    "ofdm_ctx_synchronize": (C.c_int, [_V]),
    "ofdm_ctx_trim": (C.c_int, [_V, C.POINTER(C.c_int64)]),
    "ofdm_ctx_scratch_bytes": (C.c_int, [_V, C.POINTER(C.c_int64)]),
    "ofdm_timing_enable": (C.c_int, [_V, C.c_int]),
    "ofdm_timing_query": (C.c_int, [_V, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "ofdm_timing_reset": (C.c_int, [_V]),
    "ofdm_fft64": (C.c_int, [_V, _V, _V, C.c_int64, C.c_int, C.c_int]),
    "ofdm_tx_bytes": (C.c_int, [C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "ofdm_tx_frames": (C.c_int, [_V, _V, C.c_uint64, C.c_int64, _V, _V]),
    "ofdm_set_next_tx": (C.c_int, [_V, _V, C.c_uint64, C.c_int64, _V, _V]),
    "ofdm_rx_frames": (C.c_int, [_V, _V, _V, _V, C.c_uint64, C.c_int64, _V, C.c_int, _V]),
    "ofdm_txrx_frames": (C.c_int, [_V, _V, C.c_uint64, C.c_int64, _V, _V, _V, C.c_int, _V]),
    "ofdm_rx_frames_dump": (C.c_int, [_V, _V, _V, _V, C.c_uint64, C.c_int64, _V, C.c_int, _V, _V, _V]),
    "ofdm_symbol_sweep": (C.c_int, [_V, _V, _V, C.c_int, C.c_uint64, C.c_int64, C.c_int64, _V]),
    "ofdm_set_message": (C.c_int, [_V, C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
    "ofdm_payload_frames": (C.c_int, [_V, C.c_int, C.POINTER(C.c_int32)]),
    "ofdm_transmitter": (C.c_int, [_V, C.c_int, C.c_int, C.c_int, _V, C.c_int32, C.POINTER(C.c_int32)]),
    "ofdm_transmission_over_air": (C.c_int, [_V, _V, _V, C.c_int32, C.c_double, C.c_uint64, C.c_uint64, C.c_int32]),
    "ofdm_receiver": (C.c_int, [_V, _V, _V, C.c_int, _V, _V, _V, _V]),
    "ofdm_word_length_report": (C.c_int, [_V, _V, C.c_int32, _V, C.POINTER(C.c_int32)]),
    "ofdm_frame_sweep": (C.c_int, [_V, _V, _V, _V, C.c_int, C.c_uint64, C.c_int64, _V, _V]),
}
EXPORTS = tuple(_SIGS)


class OfdmError(RuntimeError):
    pass


class Cfg(C.Structure):
    """ofdm_cfg"""
    _fields_ = [("seed", C.c_uint64), ("conv", C.c_int32), ("payload", C.c_int32), ("est", C.c_int32),
                ("noise", C.c_int32), ("channel", C.c_int32), ("data_per_frame", C.c_int32),
                ("kappa", C.c_double), ("p_ref", C.c_double)]


class RxOpts(C.Structure):
    """ofdm_rx_opts"""
    _fields_ = [("cap_len", C.c_int32), ("float_cfo", C.c_int32), ("matlab_slicer", C.c_int32),
                ("float_taps", C.c_int32), ("fixed_start", C.c_int32), ("word_stats", C.c_int32),
                ("reserved", C.c_int32 * 2)]


def make_cfg(seed: int = 0x80211A, conv: str = "c", payload: str = "random", est: str = "ls",
             noise: str = "real", channel: str = "awgn", kappa: float = 0.4980,
             p_ref: float = 52.0 / 4096.0) -> Cfg:
    return Cfg(seed, CONV[conv], PAYLOAD[payload], EST[est], NOISE[noise], CHANNEL[channel], 2, kappa, p_ref)


def wave_len(frames: int) -> int:
    """Transmitter() output length for `frames` data symbols (OFDM.c:569-612): 10 x (2 (320 + 80 D) + 20)."""
    return 10 * (2 * (320 + 80 * frames) + 20)


def capture_len(frames: int) -> int:
    """Receiver() capture, int(0.307 x waveform length) (OFDM.c:945): 3008 for D = 2."""
    return int(wave_len(frames) * 0.307)


def make_rx_opts(mode: str = "c", fixed_start: int = -1) -> RxOpts:
    """mode 'c': OFDM.c receiver (capture int(0.307 len), 3008 for the reference message; fp32 CFO,
    fp32 taps); 'matlab': IEEE_802_11_a_Code_Tester.m (capture 3000, MATLAB slicer, double taps)."""
    if mode == "c":
        return RxOpts(0, 1, 0, 1, fixed_start)
    if mode == "matlab":
        return RxOpts(3000, 0, 1, 0, fixed_start)
    raise ValueError(mode)


_LIB = None
_LIB_FILE: Path | None = None


def library_file() -> Path:
    """The shared object load_library() loaded (or would load): bench.py reads its kernels' build ids."""
    return _LIB_FILE or Path(os.environ.get("OFDM_MI355X_LIB") or LIB_PATH)


def load_library(path: Path | str | None = None) -> C.CDLL:
    """Load libofdm_mi355x.so (build it first with build_lib.build()).  Raises if absent."""
    global _LIB, _LIB_FILE
    if _LIB is not None and path is None:
        return _LIB
    # OFDM_MI355X_LIB: load a variant build (tools/build_variants.py) instead of the default
    p = Path(path or os.environ.get("OFDM_MI355X_LIB") or LIB_PATH)
    try:
        # PyTorch ships its own libamdhip64 (same SONAME).  Loading it first makes this library
        # bind to that one HIP runtime instead of starting a second one from /opt/rocm, which
        # would then see no device.
        import torch  # noqa: F401,PLC0415
    except ImportError:
        pass
    if not p.exists():
        raise OfdmError(f"{p} not found: the HIP library must be built (build_lib.build()); "
                        "there is no CPU fallback")
    lib = C.CDLL(str(p))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ofdm_abi_version() != ABI_VERSION:
        raise OfdmError(f"ABI mismatch: library {lib.ofdm_abi_version()} != {ABI_VERSION}")
    if path is None:
        _LIB, _LIB_FILE = lib, p
    return lib


def check(lib: C.CDLL, rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib.ofdm_last_error()
        raise OfdmError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
