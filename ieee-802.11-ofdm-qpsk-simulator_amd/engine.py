"""Host-side engine: one ofdm_ctx per GPU, device buffers from PyTorch (plumbing only).

Mirrors the reference's three hot-path functions (src/OFDM.c):
    Transmitter()            OFDM.c:467-618   -> Engine.transmitter() / Engine.tx_frames()
    Transmission_Over_Air()  OFDM.c:635-655   -> Engine.transmission_over_air()
    Receiver()               OFDM.c:941-1165  -> Engine.receiver() / Engine.rx_frames()
and main()'s SNR loop (OFDM.c:1187-1222) -> Engine.symbol_sweep() / Engine.frame_sweep().
All arithmetic happens in the HIP kernels of libofdm_mi355x.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi
from .abi import Cfg, RxOpts, check, load_library, make_cfg, make_rx_opts
from .fileio import decode_message


def _torch():
    import torch  # noqa: PLC0415  (device memory / streams only)
    return torch


def _ptr(t) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


class Engine:
    """A context bound to one MI355X (gfx950).  Use as a context manager or call close()."""

    def __init__(self, device: int = 0, use_torch_stream: bool = True):
        self.lib = load_library()
        self.device = device
        torch = _torch()
        if not torch.cuda.is_available():
            raise abi.OfdmError("no GPU visible: the OFDM engine runs only on gfx950")
        torch.cuda.set_device(device)
        h = C.c_void_p()
        check(self.lib, self.lib.ofdm_ctx_create(device, C.byref(h)), "ofdm_ctx_create")
        self.ctx = h
        if use_torch_stream:
            self.set_stream(torch.cuda.current_stream(device).cuda_stream)

    # ---- lifecycle -------------------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ofdm_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int | None):
        """Enqueue on this hipStream_t handle (0 / None = the null stream, PyTorch's default)."""
        check(self.lib, self.lib.ofdm_ctx_set_stream(self.ctx, C.c_void_p(stream_handle or None)), "set_stream")

    def synchronize(self):
        check(self.lib, self.lib.ofdm_ctx_synchronize(self.ctx), "synchronize")

    def trim(self) -> int:
        """Free the context's sweep scratch (ofdm_ctx_trim: up to 12 GiB of frame-sweep hand-off buffer); returns
        the bytes released.  Later sweeps allocate it again."""
        n = C.c_int64()
        check(self.lib, self.lib.ofdm_ctx_trim(self.ctx, C.byref(n)), "ctx_trim")
        return n.value

    def scratch_bytes(self) -> int:
        n = C.c_int64()
        check(self.lib, self.lib.ofdm_ctx_scratch_bytes(self.ctx, C.byref(n)), "ctx_scratch_bytes")
        return n.value

    # ---- timing ----------------------------------------------------------------------
    def timing(self, enable: bool = True):
        check(self.lib, self.lib.ofdm_timing_enable(self.ctx, int(enable)), "timing_enable")

    def timing_reset(self):
        check(self.lib, self.lib.ofdm_timing_reset(self.ctx), "timing_reset")

    def timing_query(self, kernel: int) -> tuple[float, int]:
        ms = C.c_double(); n = C.c_int64()
        check(self.lib, self.lib.ofdm_timing_query(self.ctx, kernel, C.byref(ms), C.byref(n)), "timing_query")
        return ms.value, n.value

    # ---- K1: batched 64-point transforms (device tensors, complex64 [n, 64]) -----------
    def fft64(self, x, inverse: bool = False, conv: str = "c"):
        torch = _torch()
        x = x.contiguous()
        assert x.dtype == torch.complex64 and x.shape[-1] == 64 and x.is_cuda
        out = torch.empty_like(x)
        n = x.numel() // 64
        check(self.lib, self.lib.ofdm_fft64(self.ctx, _ptr(x), _ptr(out), n, int(inverse), abi.CONV[conv]), "fft64")
        return out

    def fft64_into(self, x, out, inverse: bool = False, conv: str = "c"):
        """fft64 into a preallocated complex64 [n, 64] device tensor (no allocation; in place allowed)."""
        torch = _torch()
        assert x.dtype == torch.complex64 and out.dtype == torch.complex64 and x.is_contiguous() and out.is_contiguous()
        assert x.shape == out.shape and x.shape[-1] == 64 and x.is_cuda and out.is_cuda
        check(self.lib, self.lib.ofdm_fft64(self.ctx, _ptr(x), _ptr(out), x.numel() // 64, int(inverse), abi.CONV[conv]),
              "fft64")
        return out

    # ---- symbol mode (the per-symbol chain) ---------------------------------------------
    def tx_buffers(self, n_frames: int):
        torch = _torch()
        tb = C.c_int64(); bb = C.c_int64()
        check(self.lib, self.lib.ofdm_tx_bytes(n_frames, C.byref(tb), C.byref(bb)), "tx_bytes")
        tx = torch.empty(tb.value // 8, dtype=torch.complex64, device=f"cuda:{self.device}")
        bits = torch.empty(bb.value // 4, dtype=torch.int32, device=f"cuda:{self.device}")
        return tx, bits

    def tx_frames(self, cfg: Cfg, first_frame: int, n_frames: int, tx=None, bits=None):
        if tx is None or bits is None:
            tx, bits = self.tx_buffers(n_frames)
        check(self.lib, self.lib.ofdm_tx_frames(self.ctx, C.byref(cfg), first_frame, n_frames, _ptr(tx), _ptr(bits)),
              "tx_frames")
        return tx, bits

    def set_next_tx(self, cfg: Cfg, first_frame: int, n_frames: int, tx, bits):
        """The next rx_frames call also builds this Tx batch (ofdm_set_next_tx: fused into the packed
        receiver, else a Tx launch ahead of it on the same stream)."""
        check(self.lib, self.lib.ofdm_set_next_tx(self.ctx, C.byref(cfg), first_frame, n_frames, _ptr(tx), _ptr(bits)),
              "set_next_tx")

    def new_counters(self, n_snr: int):
        torch = _torch()
        return torch.zeros((n_snr, abi.NCOUNTERS), dtype=torch.int64, device=f"cuda:{self.device}")

    def rx_frames(self, cfg: Cfg, tx, bits, first_frame: int, n_frames: int, snr_db, counters=None):
        snr = np.ascontiguousarray(snr_db, np.float64)
        if counters is None:
            counters = self.new_counters(len(snr))
        check(self.lib, self.lib.ofdm_rx_frames(self.ctx, C.byref(cfg), _ptr(tx), _ptr(bits), first_frame, n_frames,
                                                snr.ctypes.data_as(C.c_void_p), len(snr), _ptr(counters)), "rx_frames")
        return counters

    def txrx_frames(self, cfg: Cfg, first_frame: int, n_frames: int, snr_db, tx=None, bits=None, counters=None):
        """ofdm_txrx_frames: the Tx batch (written to tx / bits) and its receiver pass in one call (one launch
        for the packed real-noise receivers)."""
        snr = np.ascontiguousarray(snr_db, np.float64)
        if tx is None or bits is None:
            tx, bits = self.tx_buffers(n_frames)
        if counters is None:
            counters = self.new_counters(len(snr))
        check(self.lib, self.lib.ofdm_txrx_frames(self.ctx, C.byref(cfg), first_frame, n_frames, _ptr(tx), _ptr(bits),
                                                  snr.ctypes.data_as(C.c_void_p), len(snr), _ptr(counters)),
              "txrx_frames")
        return tx, bits, counters

    def rx_frames_dump(self, cfg: Cfg, tx, bits, first_frame: int, n_frames: int, snr_db):
        torch = _torch()
        snr = np.ascontiguousarray(snr_db, np.float64)
        counters = self.new_counters(len(snr))
        eq = torch.zeros((len(snr), n_frames, 2, 48), dtype=torch.complex64, device=f"cuda:{self.device}")
        db = torch.zeros((len(snr), n_frames, 2, 3), dtype=torch.int32, device=f"cuda:{self.device}")
        check(self.lib, self.lib.ofdm_rx_frames_dump(self.ctx, C.byref(cfg), _ptr(tx), _ptr(bits), first_frame,
                                                     n_frames, snr.ctypes.data_as(C.c_void_p), len(snr),
                                                     _ptr(counters), _ptr(eq), _ptr(db)), "rx_frames_dump")
        return counters, eq, db

    def symbol_sweep(self, cfg: Cfg, snr_db, n_frames: int, first_frame: int = 0, chunk_frames: int = 0) -> np.ndarray:
        snr = np.ascontiguousarray(snr_db, np.float64)
        out = np.zeros((len(snr), abi.NCOUNTERS), np.int64)
        check(self.lib, self.lib.ofdm_symbol_sweep(self.ctx, C.byref(cfg), snr.ctypes.data_as(C.c_void_p), len(snr),
                                                   first_frame, n_frames, chunk_frames,
                                                   out.ctypes.data_as(C.c_void_p)), "symbol_sweep")
        return out

    # ---- frame mode (the reference's own trial) -----------------------------------------
    def set_message(self, message: str | bytes) -> int:
        """MESSAGE payload text (OFDM.c:20); returns the data symbols per frame, ceil(8 len / 96)."""
        b = message.encode("latin-1") if isinstance(message, str) else bytes(message)
        n = C.c_int32()
        check(self.lib, self.lib.ofdm_set_message(self.ctx, b, len(b), C.byref(n)), "set_message")
        return n.value

    def payload_frames(self, payload: str = "message") -> int:
        n = C.c_int32()
        check(self.lib, self.lib.ofdm_payload_frames(self.ctx, abi.PAYLOAD[payload], C.byref(n)), "payload_frames")
        return n.value

    def transmitter(self, conv: str = "c", payload: str = "message", float_taps: bool = True) -> np.ndarray:
        cap = abi.wave_len(8)
        buf = np.zeros(2 * cap, np.float32)
        n = C.c_int32()
        check(self.lib, self.lib.ofdm_transmitter(self.ctx, abi.CONV[conv], abi.PAYLOAD[payload], int(float_taps),
                                                  buf.ctypes.data_as(C.c_void_p), cap, C.byref(n)), "transmitter")
        return buf[:2 * n.value].view(np.complex64).copy()

    def transmission_over_air(self, tx: np.ndarray, snr_db: float, seed: int = 0x80211A, trial: int = 0,
                              snr_index: int = 0) -> np.ndarray:
        tx = np.ascontiguousarray(tx, np.complex64)
        out = np.zeros_like(tx)
        check(self.lib, self.lib.ofdm_transmission_over_air(self.ctx, tx.ctypes.data_as(C.c_void_p),
                                                            out.ctypes.data_as(C.c_void_p), len(tx), snr_db, seed,
                                                            trial, snr_index), "transmission_over_air")
        return out

    def receiver(self, capture: np.ndarray, mode: str = "c", payload: str = "message"):
        """Receiver() on one capture (OFDM.c:941-1182): metrics, packet_idx, bits, equalised
        subcarriers and the decoded text (Message_Generator, OFDM.c:921-939)."""
        opts = make_rx_opts(mode)
        nd = self.payload_frames(payload)
        L = opts.cap_len or abi.capture_len(nd)
        cap = np.ascontiguousarray(capture[:L], np.complex64)
        if len(cap) != L:
            raise ValueError(f"capture must hold {L} samples")
        res = np.zeros(3, np.float32); ints = np.zeros(4, np.int32)
        bits = np.zeros(96 * nd, np.int32); eq = np.zeros(2 * 48 * nd, np.float32)
        check(self.lib, self.lib.ofdm_receiver(self.ctx, cap.ctypes.data_as(C.c_void_p), C.byref(opts),
                                               abi.PAYLOAD[payload], res.ctypes.data_as(C.c_void_p),
                                               ints.ctypes.data_as(C.c_void_p), bits.ctypes.data_as(C.c_void_p),
                                               eq.ctypes.data_as(C.c_void_p)), "receiver")
        return dict(res=res, packet_idx=int(ints[0]), sync_fail=int(ints[1]), oob=int(ints[2]), frames=nd,
                    bits=bits, eq=eq.view(np.complex64).copy(), message=decode_message(bits))

    def word_length_report(self, capture: np.ndarray) -> dict:
        """Word_Optimization_Analysis (OFDM.c:38-73) of the capture's RRC matched-filter output."""
        cap = np.ascontiguousarray(capture, np.complex64)
        out = np.zeros(3, np.float32)
        bits = C.c_int32()
        check(self.lib, self.lib.ofdm_word_length_report(self.ctx, cap.ctypes.data_as(C.c_void_p), len(cap),
                                                         out.ctypes.data_as(C.c_void_p), C.byref(bits)),
              "word_length_report")
        return dict(min=float(out[0]), max=float(out[1]), max_abs=float(out[2]), bits=bits.value)

    def frame_sweep(self, cfg: Cfg, snr_db, n_trials: int, first_trial: int = 0, mode: str = "c",
                    fixed_start: int = -1, want_packet_idx: bool = False, word_stats: bool = False,
                    cap_len: int = 0):
        """cap_len 0: the mode's capture (int(0.307 len), OFDM.c:945; 3000 for 'matlab')."""
        snr = np.ascontiguousarray(snr_db, np.float64)
        out = np.zeros((len(snr), abi.NCOUNTERS), np.int64)
        pidx = np.zeros((len(snr), n_trials), np.int32) if want_packet_idx else None
        opts = make_rx_opts(mode, fixed_start)
        opts.word_stats = int(word_stats)
        if cap_len:
            opts.cap_len = int(cap_len)
        check(self.lib, self.lib.ofdm_frame_sweep(self.ctx, C.byref(cfg), C.byref(opts), snr.ctypes.data_as(C.c_void_p),
                                                  len(snr), first_trial, n_trials, out.ctypes.data_as(C.c_void_p),
                                                  None if pidx is None else pidx.ctypes.data_as(C.c_void_p)),
              "frame_sweep")
        return (out, pidx) if want_packet_idx else out


@dataclass
class SweepResult:
    snr_db: np.ndarray
    counters: np.ndarray

    @property
    def ber(self) -> np.ndarray:
        c = self.counters
        return c[:, abi.C_BIT_ERR] / np.maximum(c[:, abi.C_BITS], 1)

    @property
    def evm_pre_db(self) -> np.ndarray:
        """pooled EVM before the slicer: 10 log10(sum|z-d|^2 / sum|d|^2) (OFDM.c:1104-1126)"""
        c = self.counters
        with np.errstate(divide="ignore"):
            return 10 * np.log10(c[:, abi.C_EVM_PRE_Q] / abi.EVM_Q_SCALE / np.maximum(c[:, abi.C_EVM_TERMS], 1))

    @property
    def evm_post_db(self) -> np.ndarray:
        """pooled EVM after the slicer (OFDM.c:1128-1150); -inf when no slicer error"""
        c = self.counters
        with np.errstate(divide="ignore"):
            return 10 * np.log10(2.0 * c[:, abi.C_EVM_POST_AXIS] / np.maximum(c[:, abi.C_EVM_TERMS], 1))

    @property
    def mean_frame_evm_db(self) -> np.ndarray:
        """mean over frames of the per-frame EVM_dB the reference prints per trial (OFDM.c:1126)"""
        c = self.counters
        return c[:, abi.C_EVMDB_PRE_Q] / abi.EVM_Q_SCALE / np.maximum(c[:, abi.C_FRAMES], 1)

    @property
    def mean_frame_evm_post_db(self) -> np.ndarray:
        """mean over frames of the per-frame post-slicer EVM_dB (OFDM.c:1150); -inf when any frame
        had no slicer error (that frame's own value is -inf, OFDM.c:1148-1150)"""
        c = self.counters
        m = c[:, abi.C_EVMDB_POST_Q] / abi.EVM_Q_SCALE / np.maximum(c[:, abi.C_FRAMES], 1)
        return np.where(c[:, abi.C_EVMDB_POST_FINITE] < c[:, abi.C_FRAMES], -np.inf, m)

    @property
    def mean_finite_frame_evm_post_db(self) -> np.ndarray:
        """mean of the per-frame post-slicer EVM_dB over the frames where it is finite (frames with >= 1
        slicer error); -inf only where no frame had one.  A plottable companion of mean_frame_evm_post_db
        for many trials per point (the reference's own statistic is -inf as soon as one trial is clean)."""
        c = self.counters
        fin = c[:, abi.C_EVMDB_POST_FINITE]
        m = c[:, abi.C_EVMDB_POST_Q] / abi.EVM_Q_SCALE / np.maximum(fin, 1)
        return np.where(fin > 0, m, -np.inf)

    @property
    def sync_fail_rate(self) -> np.ndarray:
        c = self.counters
        return c[:, abi.C_SYNC_FAIL] / np.maximum(c[:, abi.C_FRAMES], 1)


__all__ = ["Engine", "SweepResult", "make_cfg", "make_rx_opts"]
