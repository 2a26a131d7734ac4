"""The frame sync kernels' lazy rules (ofdm_frame.hip: FRAME_LAZY, and frame_sync_long_kernel's round-2 skip;
DESIGN.md §4 K4b) against the reference's own Packet_Selection (src/OFDM.c:685-771, compiled in oracle/_ref) on
random captures: whenever the first detection round [0, 64 x 31) (reference message) or the first two rounds
[0, 2 x 64 x 31) (8-symbol message) decide the selection by the kernel's rule, the reference's packet_idx over
the WHOLE capture is that decision.  (The GPU tests test_lazy_capture_equals_full_evaluation and
test_long_capture_lazy_equals_full_evaluation check the kernels' lazy and full paths against each other.)"""
import ctypes as C

import numpy as np
import pytest

B1 = 64 * 31                 # round 0 of the reference capture (FRAME_LAZY_C0 = 31)
NFR = 320 + 80 * 2           # fr_len of the 2-symbol reference message
LEN_RRC_RX = 10


def corr_out(cap):
    """Packet_Detection (OFDM.c:659-683): M[i] = |sum r[i+k] r[i+k+16]|^2 / (sum |r[i+k+16]|^2)^2, k < 32"""
    lc = len(cap) - 47
    prod = cap[:-16] * cap[16:]
    pw = np.abs(cap[16:]) ** 2
    cs = np.concatenate([[0], np.cumsum(prod)])
    cp = np.concatenate([[0], np.cumsum(pw)])
    n = np.arange(lc)
    return (np.abs(cs[n + 32] - cs[n]) ** 2 / (cp[n + 32] - cp[n]) ** 2).astype(np.float32)


def lazy_decision(m, rx_start):
    """the kernel's rule: (decided, packet_idx) from round 0 alone"""
    idx = np.nonzero(m[:B1] > 0.75)[0]
    prev = np.concatenate([[-1], idx[:-1]])
    fronts = idx[(idx - prev) > 300]
    valid = [f for f in fronts if f + 230 < B1 and m[f + 230] > 0.75]
    if not valid or valid[0] >= fronts.max():
        return False, None
    f = valid[0]
    gen = 4 * (((rx_start + B1 + 46) >> 2) + 1) - rx_start          # capture samples generated before round 0
    if f + LEN_RRC_RX + 1 + 2 * (NFR - 1) + 10 >= gen:
        return False, None
    return True, int(f) + LEN_RRC_RX + 1


@pytest.mark.parametrize("snr_db", [0.0, 6.0, 9.0, 12.0, 16.0, 30.0])
def test_round0_decision_is_the_references(reflib, snr_db):
    wave = reflib.waveform().astype(np.complex128)
    L = int(0.307 * len(wave))
    rng = np.random.default_rng(int(snr_db * 10) + 1)
    sigma = np.sqrt(np.mean(np.abs(wave) ** 2) / 10 ** (snr_db / 10))
    decided = 0
    for _ in range(400):
        s = int(rng.integers(0, len(wave) - L))
        cap = wave[s:s + L] + sigma * rng.standard_normal(L)        # real-only AWGN (D7)
        m = corr_out(cap)
        ok, p = lazy_decision(m, s)
        if ok:
            decided += 1
            ref = reflib.lib.ref_packet_selection(m.ctypes.data_as(C.c_void_p), len(m))
            assert ref == p, (snr_db, s)
    if snr_db >= 12:
        assert decided > 0.6 * 400                                  # the rule does skip work where sync works


def rounds_decision(m, limit):
    """frame_sync_long_kernel's rule: (decided, packet_idx) from the positions below `limit` alone"""
    idx = np.nonzero(m[:limit] > 0.75)[0]
    if len(idx) == 0:
        return False, None
    prev = np.concatenate([[-1], idx[:-1]])
    fronts = idx[(idx - prev) > 300]
    valid = [f for f in fronts if f + 230 < limit and m[f + 230] > 0.75]
    if not valid or valid[0] >= fronts.max():
        return False, None
    return True, int(valid[0]) + LEN_RRC_RX + 1


def packet_selection(m, thr=0.75):
    """Packet_Selection (OFDM.c:685-771) over the whole of M with the threshold as a parameter: the first front
    (a crossing more than 300 positions past the previous one) but the last whose M[front + 230] crosses too ->
    front + len_RRC_rx + 1; 0 when none does.  tests/test_gpu_frame.py moves `thr` to show that a packet_idx on
    which the GPU and the oracle differ sits on the threshold."""
    idx = np.nonzero(m > thr)[0]
    prev = np.concatenate([[-1], idx[:-1]])
    fronts = idx[(idx - prev) > 300]
    for f in fronts[:-1]:
        if f + 230 < len(m) and m[f + 230] > thr:
            return int(f) + LEN_RRC_RX + 1
    return 0


@pytest.mark.parametrize("snr_db", [0.0, 6.0, 9.0, 12.0, 30.0])
def test_packet_selection_helper_is_the_references(reflib, snr_db):
    wave = reflib.waveform().astype(np.complex128)
    L = int(0.307 * len(wave))
    rng = np.random.default_rng(int(snr_db * 10) + 7)
    sigma = np.sqrt(np.mean(np.abs(wave) ** 2) / 10 ** (snr_db / 10))
    for _ in range(200):
        s = int(rng.integers(0, len(wave) - L))
        m = corr_out(wave[s:s + L] + sigma * rng.standard_normal(L))
        ref = reflib.lib.ref_packet_selection(m.ctypes.data_as(C.c_void_p), len(m))
        assert packet_selection(m) == ref, (snr_db, s)


@pytest.mark.parametrize("snr_db", [0.0, 6.0, 10.0, 16.0, 30.0])
def test_long_frames_two_round_decision_is_the_references(oracle, reflib, snr_db):
    msg = (b"lazy rounds for the long-capture kernel: two frame periods decide most trials. " * 2)[:96]
    wave = oracle.frame_waveform(oracle.message_bits(msg)).astype(np.complex128)     # the oracle's message is untouched
    L = int(0.307 * len(wave))
    assert L == 5955
    rng = np.random.default_rng(int(snr_db * 10) + 3)
    sigma = np.sqrt(np.mean(np.abs(wave) ** 2) / 10 ** (snr_db / 10))
    decided = 0
    for _ in range(150):
        s = int(rng.integers(0, len(wave) - L))
        cap = wave[s:s + L] + sigma * rng.standard_normal(L)        # real-only AWGN (D7)
        m = corr_out(cap)
        ok, p = rounds_decision(m, 2 * B1)
        if ok:
            decided += 1
            ref = reflib.lib.ref_packet_selection(m.ctypes.data_as(C.c_void_p), len(m))
            assert ref == p, (snr_db, s)
    if snr_db >= 16:
        assert decided > 0.8 * 150                                  # round 2 is skipped where sync works
