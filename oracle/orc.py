"""ctypes front-ends for the oracle libraries (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
# OFDM_ORACLE_SO / OFDM_REF_SO: other builds of the same sources (tools/sanitize.py's ASan builds in _asan/)
ORACLE_SO = Path(os.environ.get("OFDM_ORACLE_SO", ORACLE_DIR / "_lib" / "liboracle.so"))
REF_SO = Path(os.environ.get("OFDM_REF_SO", ORACLE_DIR / "_ref" / "libofdm_ref.so"))
REF_SRC = Path(os.environ.get("OFDM_REF_SRC", "/root/reference/src/OFDM.c"))

NCOUNTERS = 16
CONV = {"c": 0, "matlab": 1}
PAYLOAD = {"random": 0, "message": 1, "tester": 2}
EST = {"ls": 0, "ideal": 1}
NOISE = {"real": 0, "complex": 1, "none": 2}
CHANNEL = {"awgn": 0, "rayleigh4": 1}


def build_oracle() -> Path:
    subprocess.run(["make", "-s", "oracle"], cwd=ORACLE_DIR, check=True)
    return ORACLE_SO


def build_ref() -> Path | None:
    """Compile the reference (only where its source exists: this container, not the GPU box)."""
    if not REF_SRC.exists():
        return REF_SO if REF_SO.exists() else None
    subprocess.run(["make", "-s", "ref", f"REF_SRC={REF_SRC}"], cwd=ORACLE_DIR, check=True)
    return REF_SO


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class _Cfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("conv", C.c_int), ("payload", C.c_int), ("est", C.c_int),
                ("noise", C.c_int), ("channel", C.c_int), ("data_per_frame", C.c_int),
                ("kappa", C.c_double), ("p_ref", C.c_double)]


class _RxOpts(C.Structure):
    _fields_ = [("cap_len", C.c_int), ("float_cfo", C.c_int), ("matlab_slicer", C.c_int),
                ("float_taps", C.c_int)]


class _RxInfo(C.Structure):
    _fields_ = [("packet_idx", C.c_int), ("len_corr", C.c_int), ("sync_fail", C.c_int),
                ("oob", C.c_int), ("res", C.c_double * 3), ("cfo", C.c_double * 2)]


def c2i(z: np.ndarray) -> np.ndarray:
    """complex -> interleaved float64"""
    z = np.ascontiguousarray(z, dtype=np.complex128)
    return z.view(np.float64)


def i2c(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64).view(np.complex128)


class Oracle:
    """Our double-precision CPU restatement (oracle/ofdm_oracle.c)."""

    def __init__(self, path: Path | None = None):
        path = Path(path or ORACLE_SO)
        if not path.exists():
            build_oracle()
        self.lib = C.CDLL(str(path))
        L = self.lib
        L.orc_symbol_sweep.argtypes = [C.POINTER(_Cfg), C.c_void_p, C.c_int, C.c_uint64, C.c_uint64,
                                       C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_frame_sweep.argtypes = [C.POINTER(_Cfg), C.POINTER(_RxOpts), C.c_void_p, C.c_int,
                                      C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
        L.orc_time_symbol_sweep.argtypes = [C.POINTER(_Cfg), C.c_void_p, C.c_int, C.c_uint64, C.c_void_p]
        L.orc_time_symbol_sweep.restype = C.c_double
        L.orc_receiver_frame.argtypes = [C.c_void_p, C.POINTER(_RxOpts), C.c_void_p, C.c_int] + \
            [C.c_void_p] * 8 + [C.POINTER(_RxInfo)]
        L.orc_frame_waveform.restype = C.c_int
        L.orc_message_bits.restype = C.c_int
        L.orc_set_message.restype = C.c_int
        L.orc_word_length.restype = C.c_int
        L.orc_word_length.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.orc_set_message.argtypes = [C.c_char_p, C.c_int]
        self._frames = 2

    def word_length(self, capture: np.ndarray, float_taps: bool = True):
        """Word_Optimization_Analysis of the RRC-filtered capture -> (min, max, max_abs, bits)."""
        out = np.zeros(3)
        cap = c2i(np.asarray(capture))
        bits = self.lib.orc_word_length(_p(cap), len(capture), int(float_taps), _p(out))
        return out[0], out[1], out[2], bits

    def set_message(self, msg: bytes) -> int:
        """MESSAGE payload text used by the sweeps (default OFDM.c:20); returns data symbols per frame."""
        n = self.lib.orc_set_message(bytes(msg), len(msg))
        if n < 0:
            raise ValueError("message length must be 1..96")
        self._frames = n
        return n

    # ---- small helpers -------------------------------------------------------
    @staticmethod
    def cfg(seed=0x80211A, conv="c", payload="random", est="ls", noise="real", channel="awgn",
            kappa=0.4980, p_ref=52.0 / 4096.0) -> _Cfg:
        return _Cfg(seed, CONV[conv], PAYLOAD[payload], EST[est], NOISE[noise], CHANNEL[channel], 2,
                    kappa, p_ref)

    @staticmethod
    def rx_opts(mode="c", frames: int = 2) -> _RxOpts:
        if mode == "c":   # int(0.307 x waveform length) (OFDM.c:945): 3008 for 2 data symbols
            return _RxOpts(int(10 * (2 * (320 + 80 * frames) + 20) * 0.307), 1, 0, 1)
        return _RxOpts(3000, 0, 1, 0)     # MATLAB Tester (Tester.m:151-152)

    def philox(self, ctr, key) -> np.ndarray:
        c = np.asarray(ctr, np.uint32); k = np.asarray(key, np.uint32); o = np.zeros(4, np.uint32)
        self.lib.orc_philox4x32_10(_p(c), _p(k), _p(o))
        return o

    def gauss4(self, ctr, key) -> np.ndarray:
        c = np.asarray(ctr, np.uint32); k = np.asarray(key, np.uint32); o = np.zeros(4, np.float64)
        self.lib.orc_gauss4(_p(c), _p(k), _p(o))
        return o

    def fft64(self, x: np.ndarray) -> np.ndarray:
        i = c2i(x); o = np.zeros(128)
        self.lib.orc_fft64(_p(i), _p(o))
        return i2c(o)

    def ifft64(self, X: np.ndarray, conv="c") -> np.ndarray:
        i = c2i(X); o = np.zeros(128)
        self.lib.orc_ifft64(_p(i), _p(o), CONV[conv])
        return i2c(o)

    def message_bits(self, msg: bytes) -> np.ndarray:
        nf = (8 * len(msg) + 95) // 96
        b = np.zeros(96 * nf, np.int32)
        buf = (C.c_ubyte * len(msg)).from_buffer_copy(msg)
        self.lib.orc_message_bits(buf, len(msg), _p(b))
        return b

    def tester_bits(self) -> np.ndarray:
        b = np.zeros(192, np.int32)
        self.lib.orc_tester_bits(_p(b))
        return b

    def data_symbol(self, bits96, conv="c") -> np.ndarray:
        b = np.ascontiguousarray(bits96, np.int32); o = np.zeros(160)
        self.lib.orc_data_symbol(_p(b), CONV[conv], _p(o))
        return i2c(o)

    def preambles(self, conv="c"):
        s = np.zeros(320); l = np.zeros(320); f = np.zeros(128)
        self.lib.orc_preambles(CONV[conv], _p(s), _p(l), _p(f))
        return i2c(s), i2c(l), i2c(f)

    def rrc_taps(self, float_rounded=True) -> np.ndarray:
        h = np.zeros(21)
        self.lib.orc_rrc_taps(int(float_rounded), _p(h))
        return h

    def frame_waveform(self, bits, conv="c", float_taps=True, reps=10) -> np.ndarray:
        b = np.ascontiguousarray(bits, np.int32)
        nf = len(b) // 96
        n = (2 * (320 + 80 * nf) + 20) * reps
        o = np.zeros(2 * n)
        self.lib.orc_frame_waveform(_p(b), nf, CONV[conv], int(float_taps), reps, _p(o))
        return i2c(o)

    def receiver_frame(self, capture: np.ndarray, truth_bits, mode="c", dumps=False):
        tb = np.ascontiguousarray(truth_bits, np.int32)
        nf = len(tb) // 96
        opts = self.rx_opts(mode, nf)
        cap = c2i(capture[:opts.cap_len])
        fsz = 320 + 80 * nf
        info = _RxInfo()
        bits = np.zeros(96 * nf, np.int32)
        d = None
        if dumps:
            lc = opts.cap_len - 47
            d = dict(corr=np.zeros(lc), rxframe=np.zeros(2 * fsz), coarse=np.zeros(2 * fsz),
                     fine=np.zeros(2 * fsz), H=np.zeros(128), Yf=np.zeros(128 * nf),
                     nopilot=np.zeros(96 * nf))
            ptrs = [_p(d[k]) for k in ("corr", "rxframe", "coarse", "fine", "H", "Yf", "nopilot")]
        else:
            ptrs = [None] * 7
        self.lib.orc_receiver_frame(_p(cap), C.byref(opts), _p(tb), nf, *ptrs, _p(bits), C.byref(info))
        out = dict(bits=bits, packet_idx=info.packet_idx, sync_fail=info.sync_fail, oob=info.oob,
                   res=np.array(info.res[:]), cfo=np.array(info.cfo[:]))
        if d is not None:
            out.update({k: (v if k == "corr" else i2c(v)) for k, v in d.items()})
        return out

    def symbol_sweep(self, cfg: _Cfg, snr_db, first_frame=0, n_frames=64, dumps=False):
        snr = np.ascontiguousarray(snr_db, np.float64)
        cnt = np.zeros((len(snr), NCOUNTERS), np.int64)
        eq = np.zeros((len(snr), n_frames, 2, 48, 2)) if dumps else None
        bits = np.zeros((len(snr), n_frames, 2, 96), np.int32) if dumps else None
        self.lib.orc_symbol_sweep(C.byref(cfg), _p(snr), len(snr), first_frame, n_frames, _p(cnt),
                                  _p(eq), _p(bits))
        if dumps:
            return cnt, eq[..., 0] + 1j * eq[..., 1], bits
        return cnt

    def frame_sweep(self, cfg: _Cfg, snr_db, first_trial=0, n_trials=16, mode="c", dump_pidx=False):
        snr = np.ascontiguousarray(snr_db, np.float64)
        cnt = np.zeros((len(snr), NCOUNTERS), np.int64)
        pidx = np.zeros((len(snr), n_trials), np.int32) if dump_pidx else None
        opts = self.rx_opts(mode, self._frames if cfg.payload == PAYLOAD["message"] else 2)
        self.lib.orc_frame_sweep(C.byref(cfg), C.byref(opts), _p(snr), len(snr), first_trial, n_trials,
                                 _p(cnt), _p(pidx))
        return (cnt, pidx) if dump_pidx else cnt

    def time_symbol_sweep(self, cfg: _Cfg, snr_db, n_frames):
        snr = np.ascontiguousarray(snr_db, np.float64)
        cnt = np.zeros((len(snr), NCOUNTERS), np.int64)
        t = self.lib.orc_time_symbol_sweep(C.byref(cfg), _p(snr), len(snr), n_frames, _p(cnt))
        return t, cnt


class RefLib:
    """The unmodified reference OFDM.c behind oracle/ref_harness.c (hooks: main, rand)."""

    def __init__(self, path: Path | None = None):
        path = Path(path or REF_SO)
        if not path.exists():
            raise FileNotFoundError(f"{path} missing: run oracle/Makefile 'ref' where the reference exists")
        self.lib = C.CDLL(str(path))
        L = self.lib
        L.ref_init.restype = C.c_int
        L.ref_time_trials.restype = C.c_double
        L.ref_time_trials.argtypes = [C.c_float, C.c_int, C.c_void_p]
        L.ref_mc_trials.restype = C.c_double
        L.ref_mc_trials.argtypes = [C.c_float, C.c_int, C.c_void_p]
        L.ref_toa.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_int]
        L.ref_trial.argtypes = [C.c_float, C.c_void_p]
        L.ref_seed.argtypes = [C.c_uint64]
        L.ref_seed_bits.argtypes = [C.c_uint64]
        L.ref_packet_selection.restype = C.c_int
        L.ref_time_symbol_chain.restype = C.c_double
        L.ref_time_symbol_chain.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.ref_time_fft.restype = C.c_double
        L.ref_time_fft.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        self.n = L.ref_init()

    def waveform(self) -> np.ndarray:
        o = np.zeros(2 * self.n, np.float32)
        self.lib.ref_tx_copy(_p(o), self.n)
        return o.view(np.complex64).copy()

    def globals(self):
        bits = np.zeros(192, np.float32); pm = np.zeros(192, np.float32); lf = np.zeros(128, np.float32)
        dims = np.zeros(4, np.int32)
        self.lib.ref_globals(_p(bits), _p(pm), _p(lf), _p(dims))
        return dict(bits=bits.astype(np.int32), payload_mod=pm.view(np.complex64).copy(),
                    ltf_freq=lf.view(np.complex64).copy(), dims=dims)

    def rrc_taps(self) -> np.ndarray:
        h = np.zeros(21, np.float32)
        self.lib.ref_rrc_taps(_p(h))
        return h

    def fft(self, x: np.ndarray) -> np.ndarray:
        i = np.ascontiguousarray(x, np.complex64); o = np.zeros_like(i)
        self.lib.ref_fft(_p(i), _p(o), len(i))
        return o

    def ifft(self, X: np.ndarray) -> np.ndarray:
        i = np.ascontiguousarray(X, np.complex64); o = np.zeros_like(i)
        self.lib.ref_ifft(_p(i), _p(o), len(i))
        return o

    def time_fft(self, n_transforms: int, inverse: bool = False, n_vectors: int = 1024, seed: int = 1):
        """n_transforms calls of the reference's fft() / ifft() on 64 samples (ref_harness.c ref_time_fft) over
        n_vectors distinct seeded inputs: (seconds, checksum)."""
        x = np.random.default_rng(seed).standard_normal((n_vectors, 128)).astype(np.float32)
        chk = C.c_double()
        t = self.lib.ref_time_fft(_p(x), int(n_vectors), int(n_transforms), int(inverse), C.byref(chk))
        return t, chk.value

    def channel_estimation(self, frame480: np.ndarray) -> np.ndarray:
        """Channel_Estimation (OFDM.c:830-850) on a 480-sample symbol-rate frame -> H[64]."""
        i = np.ascontiguousarray(frame480, np.complex64); o = np.zeros(64, np.complex64)
        self.lib.ref_channel_estimation(_p(i), _p(o))
        return o

    def receiver_stages(self, ota: np.ndarray, rx_start: int):
        ota = np.ascontiguousarray(ota, np.complex64)
        nf = 2
        d = dict(corr=np.zeros(2961, np.float32), rxframe=np.zeros(480, np.complex64),
                 coarse=np.zeros(480, np.complex64), fine=np.zeros(480, np.complex64),
                 H=np.zeros(64, np.complex64), Yf=np.zeros(64 * nf, np.complex64),
                 nopilot=np.zeros(48 * nf, np.complex64), bits=np.zeros(96 * nf, np.float32),
                 res=np.zeros(3, np.float32), ints=np.zeros(4, np.int32))
        keys = ("corr", "rxframe", "coarse", "fine", "H", "Yf", "nopilot", "bits", "res", "ints")
        self.lib.ref_receiver_stages(_p(ota), len(ota), int(rx_start), *[_p(d[k]) for k in keys])
        d["bits"] = d["bits"].astype(np.int32)
        d["packet_idx"] = int(d["ints"][0])
        return d

    def receiver(self, ota: np.ndarray, rx_start: int) -> np.ndarray:
        """Receiver() itself; its rand() capture offset is scripted to rx_start (OFDM.c:949)."""
        ota = np.ascontiguousarray(ota, np.complex64)
        script = (C.c_int * 1)(int(rx_start))
        self._script = script
        self.lib.ref_script(script, 1)
        res = np.zeros(3, np.float32)
        self.lib.ref_receiver(_p(ota), len(ota), _p(res))
        self.lib.ref_seed(C.c_uint64(0x80211A))
        return res

    def toa(self, tx: np.ndarray, snr_db: float, seed: int) -> np.ndarray:
        tx = np.ascontiguousarray(tx, np.complex64); o = np.zeros_like(tx)
        self.lib.ref_seed(C.c_uint64(seed))
        self.lib.ref_toa(_p(tx), _p(o), C.c_float(snr_db), len(tx))
        return o

    def time_trials(self, snr_db: float, n_trials: int, seed: int = 0x80211A):
        acc = np.zeros(3, np.float64)
        self.lib.ref_seed(C.c_uint64(seed))
        t = self.lib.ref_time_trials(C.c_float(snr_db), int(n_trials), _p(acc))
        return t, acc

    def mc_trials(self, snr_db: float, n_trials: int, seed: int):
        """time_trials with per-trial statistics (ref_harness.c ref_mc_trials): (seconds, acc8) with
        acc8 = [sum EVM_dB, sum EVM_AGC_dB, sum BER, sum BER^2, #BER>0, #BER>=1/4, sum EVM_dB^2,
        #finite EVM_AGC_dB]."""
        acc = np.zeros(8, np.float64)
        self.lib.ref_seed(C.c_uint64(seed))
        t = self.lib.ref_mc_trials(C.c_float(snr_db), int(n_trials), _p(acc))
        return t, acc

    def time_symbol_chain(self, snr_db, n_frames: int, rayleigh: bool = False, seed: int = 0x80211A,
                          ideal: bool = False):
        """The genie symbol chain of the GPU sweep built from the reference's own stage functions
        (ref_harness.c ref_time_symbol_chain); returns (seconds, [bit errors, bits, sum|z-d|^2]).
        ideal: the known channel instead of the per-SNR LTF estimate (config c2)."""
        snr = np.ascontiguousarray(snr_db, np.float32)
        acc = np.zeros(3, np.float64)
        self.lib.ref_seed(C.c_uint64(seed))
        t = self.lib.ref_time_symbol_chain(_p(snr), len(snr), int(n_frames), int(rayleigh) | 2 * int(ideal),
                                            _p(acc))
        return t, acc

    def symbol_chain_stats(self, snr_db: float, n_frames: int, seed: int):
        """The same chain at one SNR point for a golden fixture (gen_golden.py --only chain): noise and payload
        streams seeded by `seed`; returns [bit errors, bits, sum|z-d|^2, sum of per-frame bit errors^2,
        frames with an error]."""
        snr = np.ascontiguousarray([snr_db], np.float32)
        acc = np.zeros(5, np.float64)
        self.lib.ref_seed(C.c_uint64(seed))
        self.lib.ref_seed_bits(C.c_uint64(0x9E3779B97F4A7C15 ^ (seed * 0x2545F4914F6CDD1D % (1 << 64))))
        self.lib.ref_time_symbol_chain(_p(snr), 1, int(n_frames), 4, _p(acc))
        return acc
