"""GPU parity of frame mode: Transmitter(), Transmission_Over_Air(), Receiver()
and the batched frame sweep, against the compiled reference's golden outputs, the MATLAB
known-answer vector and the oracle."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, load_golden, normwise

pytestmark = pytest.mark.gpu


def test_transmitter_vs_reference(engine):
    g = load_golden("tx_waveform.npz")
    w = engine.transmitter("c", "message")
    assert w.shape == (9800,)
    assert normwise(w, g["waveform"]) < 2e-6


def test_transmitter_matlab_tester_vs_oracle(engine, oracle):
    w = engine.transmitter("matlab", "tester")
    ref = oracle.frame_waveform(oracle.tester_bits(), "matlab", False, 10)
    assert normwise(w, ref) < 2e-6


def test_receiver_vs_reference_stages(engine):
    """Injected-noise captures through the reference's Receiver() (tests/golden/rx_stages.npz)."""
    g = load_golden("rx_stages.npz")
    w = load_golden("tx_waveform.npz")["waveform"]
    for k in range(len(g["snr"])):
        rs = int(g["rx_start"][k])
        cap = (w[rs:rs + 3008] + g["noise"][k]).astype(np.complex64)
        o = engine.receiver(cap, "c", "message")
        assert o["packet_idx"] == int(g["packet_idx"][k]), k
        ref_eq = g["nopilot"][k]
        assert normwise(o["eq"], ref_eq) < 1e-4, k
        near = np.repeat((np.abs(ref_eq.real) < 1e-4) | (np.abs(ref_eq.imag) < 1e-4), 2)
        assert not np.any((o["bits"] != g["bits"][k]) & ~near), k
        assert o["res"][2] == pytest.approx(float(g["res"][k][2]), abs=1e-6)
        assert o["res"][0] == pytest.approx(float(g["res"][k][0]), abs=2e-3)


def test_matlab_known_answer(engine, tmp_path):
    """data/Matlab_Output.txt (D6): MATLAB ifft convention, Tester payload, noiseless, capture [0,3000)."""
    kat = load_golden("matlab_output.npz")["bits"]
    w = engine.transmitter("matlab", "tester")
    o = engine.receiver(w[:3000], "matlab", "tester")
    assert np.array_equal(o["bits"][:96], kat)
    # the file compare_double.py diffs against Matlab_Output.txt
    import ofdm_pkg
    pkg = ofdm_pkg.load()
    from ofdm_amd import fileio
    fileio.write_bits_file(o["bits"][:96], tmp_path / "Code_Output.txt")
    got = np.array([float(t) for t in (tmp_path / "Code_Output.txt").read_text().split()])
    assert np.max(np.abs(got - kat)) <= 1e-6
    assert pkg is not None
    # keep the file for the container's unmodified compare_double.py run (tests/test_host.py), which
    # reads the committed copy tests/golden/gpu_kat_Code_Output.txt
    import os
    out = os.environ.get("OFDM_KAT_OUT")
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            f.write((tmp_path / "Code_Output.txt").read_text())


def test_c_receiver_tester_payload(engine):
    # with the Tester payload the C receiver makes 13/192 errors (11 in frame 1)
    w = engine.transmitter("c", "tester")
    o = engine.receiver(w[:3008], "c", "tester")
    tb = np.array([(0x41 >> (7 - b)) & 1 for b in range(8)] * 11 + [(0x20 >> (7 - b)) & 1 for b in range(8)], np.int32)
    truth = np.concatenate([tb, tb])
    assert int(np.sum(o["bits"] != truth)) == 13


def test_transmission_over_air_statistics(engine):
    w = engine.transmitter("c", "message")
    P = float(np.mean(np.abs(w.astype(np.complex128)) ** 2))
    for snr in (0.0, 10.0):
        ota = engine.transmission_over_air(w, snr, seed=5, trial=3, snr_index=1)
        n = (ota - w).astype(np.complex128)
        assert np.array_equal(ota.imag, w.imag)                    # real-only noise (D7)
        var = np.var(n.real)
        assert abs(var / (P / 10 ** (snr / 10)) - 1) < 0.05
        ota2 = engine.transmission_over_air(w, snr, seed=5, trial=3, snr_index=1)
        assert np.array_equal(ota, ota2)                           # counter-based: reproducible


def test_sweep_trial_equals_receiver_of_ota(engine, oracle, pkg):
    """trial t of the batched sweep == Receiver(Transmission_Over_Air(wave)[rx_start:]) (same streams)."""
    w = engine.transmitter("c", "message")
    cfg = pkg.make_cfg(payload="message")
    snrs = [8.0, 9.0]
    n = 40
    cnt, pidx = engine.frame_sweep(cfg, snrs, n, first_trial=100, want_packet_idx=True)
    for q in (0, 1):
        for t in (100, 117, 139):
            rs = int(oracle.philox([t, 0, 0, 0x5B000000 | q], [0x80211A, 0])[0] % (9800 - 3008))
            ota = engine.transmission_over_air(w, snrs[q], seed=0x80211A, trial=t, snr_index=q)
            o = engine.receiver(ota[rs:rs + 3008], "c", "message")
            assert o["packet_idx"] == pidx[q, t - 100]


def test_frame_sweep_vs_oracle(engine, oracle, pkg):
    snrs = [6.0, 8.0, 10.0, 14.0]
    n = 300
    g, gp = engine.frame_sweep(pkg.make_cfg(payload="message"), snrs, n, want_packet_idx=True)
    o, op = oracle.frame_sweep(oracle.cfg(payload="message"), snrs, 0, n, "c", dump_pidx=True)
    agree = np.mean(gp == op)
    assert agree > 0.995, agree
    # every packet_idx on which they differ sits on Packet_Selection's 0.75 threshold (fp32 sliding sums on the GPU,
    # double ones in the oracle), not on a different rule
    from conftest import off_threshold_pidx_mismatches  # noqa: PLC0415
    w = engine.transmitter("c", "message")
    assert off_threshold_pidx_mismatches(engine, oracle, w, snrs, gp, op, 3008) == []
    assert np.array_equal(g[:, 0], o[:, 0])
    assert np.all(np.abs(g[:, 3] - o[:, 3]) <= 96 * np.sum(gp != op, axis=1) + 2)
    assert np.all(np.abs(g[:, 5] - o[:, 5]) <= np.sum(gp != op, axis=1))


def test_lazy_capture_equals_full_evaluation(engine, pkg, monkeypatch):
    """The sync kernel generates the rest of a capture and runs its second detection round only when the
    first round (positions [0, 1984) of the reference capture) does not decide Packet_Selection
    (OFDM.c:685-771) or the matched filter would read past the generated samples.  Every counter and every
    packet_idx must equal the full evaluation's (OFDM_FRAME_NO_LAZY) on the same streams, over the bench's
    SNR grid and for an 8-symbol message (two long detection rounds)."""
    snrs = np.arange(0.0, 31.0, 2.0)
    cfg = pkg.make_cfg(payload="message")
    lazy, lp = engine.frame_sweep(cfg, snrs, 3000, want_packet_idx=True)
    monkeypatch.setenv("OFDM_FRAME_NO_LAZY", "1")
    full, fp = engine.frame_sweep(cfg, snrs, 3000, want_packet_idx=True)
    assert np.array_equal(lp, fp)
    assert np.array_equal(lazy, full)
    assert np.mean(lp[8:] > 0) > 0.99                         # >= 16 dB: nearly every trial synchronises
    monkeypatch.delenv("OFDM_FRAME_NO_LAZY")
    msg = (b"lazy capture, eight data symbols. " * 3)[:96]
    monkeypatch.setenv("OFDM_FRAME_NO_LONG", "1")     # the generic kernel's lazy path (the long kernel has none)
    with pkg.Engine(0) as e8:
        assert e8.set_message(msg) == 8
        cfg8 = pkg.make_cfg(payload="message")
        lazy8, lp8 = e8.frame_sweep(cfg8, snrs[::3], 500, want_packet_idx=True)
        monkeypatch.setenv("OFDM_FRAME_NO_LAZY", "1")
        full8, fp8 = e8.frame_sweep(cfg8, snrs[::3], 500, want_packet_idx=True)
    assert np.array_equal(lp8, fp8)
    assert np.array_equal(lazy8, full8)


@pytest.mark.parametrize("no_lazy", [False, True])
def test_fixed_geometry_kernel_equals_generic(engine, pkg, monkeypatch, no_lazy):
    """The reference message's sweep (2 data symbols, the 3008-sample capture of OFDM.c:945) runs the sync
    kernel instantiated with that geometry as compile-time constants; OFDM_FRAME_GENERIC=1 runs the generic
    instantiation (every size from the arguments, as for other messages and the parity dumps).  Every counter
    and packet_idx is identical, lazy or full evaluation, over the bench's SNR grid."""
    snrs = np.arange(0.0, 31.0, 2.0)
    cfg = pkg.make_cfg(payload="message")
    if no_lazy:
        monkeypatch.setenv("OFDM_FRAME_NO_LAZY", "1")
    fixed, fp = engine.frame_sweep(cfg, snrs, 4000, want_packet_idx=True, first_trial=77)
    monkeypatch.setenv("OFDM_FRAME_GENERIC", "1")
    gen, gp = engine.frame_sweep(cfg, snrs, 4000, want_packet_idx=True, first_trial=77)
    assert np.array_equal(fp, gp)
    assert np.array_equal(fixed, gen)
    assert fixed[0, 0] == 4000


def test_long_message_one_wave_blocks_equal_four_wave_blocks(pkg, monkeypatch):
    """An 8-symbol message's 5955-sample captures take 24 KB of LDS per wave in the generic sync kernel: one
    four-wave block fits per CU, five one-wave blocks would (measured slower, see run_frame_chunk).  The
    one-wave instantiation (OFDM_FRAME_BLOCK1=1) gives every counter and packet_idx of the four-wave one (both with
    the long-capture kernel switched off, OFDM_FRAME_NO_LONG=1)."""
    snrs = np.array([4.0, 10.0, 16.0, 30.0])
    msg = (b"one-wave blocks for long messages " * 3)[:96]
    monkeypatch.setenv("OFDM_FRAME_NO_LONG", "1")
    with pkg.Engine(0) as e8:
        assert e8.set_message(msg) == 8
        cfg8 = pkg.make_cfg(payload="message")
        four, p4 = e8.frame_sweep(cfg8, snrs, 3000, want_packet_idx=True)
        monkeypatch.setenv("OFDM_FRAME_BLOCK1", "1")
        one, p1 = e8.frame_sweep(cfg8, snrs, 3000, want_packet_idx=True)
    assert np.array_equal(p1, p4)
    assert np.array_equal(one, four)
    assert np.mean(p1[2:] > 0) > 0.99


@pytest.mark.parametrize("msg_len", [96, 80, 49])
def test_long_capture_kernel_equals_generic(pkg, monkeypatch, msg_len):
    """Frames of >= 5 data symbols (captures > 4,100 samples) run frame_sync_long_kernel: the capture in a per-wave
    ring of 2,976 floats (+ mirror) generated a detection round at a time, the part of the matched-filter window the
    ring does not hold generated again, fr[] over the region.  Every counter and packet_idx equals the generic
    kernel's (OFDM_FRAME_NO_LONG=1), over the bench's SNR grid, for 8-, 7- and 5-symbol messages.  Every long capture
    has three detection rounds (its Lc > 2 x 1,984 positions); the 5-symbol 4,482-sample capture's last round is only
    467 positions long.  Chunked long sweeps (chunk starts off the SNR grid) are
    test_frame_sweep_nomem_halving_and_nonzero_q0[message8]."""
    snrs = np.arange(0.0, 31.0, 2.0)
    msg = (b"The long-capture kernel keeps two pieces of the capture resident per wave. " * 2)[:msg_len]
    with pkg.Engine(0) as e:
        nd = e.set_message(msg)
        assert nd == -(-8 * msg_len // 96) and nd >= 5
        cfg = pkg.make_cfg(payload="message")
        lng, lp = e.frame_sweep(cfg, snrs, 1500, want_packet_idx=True, first_trial=3)
        monkeypatch.setenv("OFDM_FRAME_NO_LONG", "1")
        gen, gp = e.frame_sweep(cfg, snrs, 1500, want_packet_idx=True, first_trial=3)
        monkeypatch.delenv("OFDM_FRAME_NO_LONG")
    assert np.array_equal(lp, gp)
    assert np.array_equal(lng, gen)
    assert lng[0, 0] == 1500 and np.mean(lp[-4:] > 0) > 0.99       # high SNR: nearly every trial synchronises
    assert lng[-1, 3] == 0                                           # 30 dB: error-free


def test_long_capture_lazy_equals_full_evaluation(pkg, monkeypatch):
    """frame_sync_long_kernel skips detection round 2 and its capture samples when rounds 0 and 1 decide
    Packet_Selection (their least valid front has a later front in them).  Every counter and packet_idx equals the
    evaluation of every round (OFDM_FRAME_NO_LAZY=1), over the bench's SNR grid, where low-SNR items need round 2
    (noise fronts) and high-SNR ones do not."""
    snrs = np.arange(0.0, 31.0, 2.0)
    msg = (b"lazy rounds for the long-capture kernel: two frame periods decide most trials. " * 2)[:96]
    with pkg.Engine(0) as e:
        assert e.set_message(msg) == 8
        cfg = pkg.make_cfg(payload="message")
        lz, lp = e.frame_sweep(cfg, snrs, 1500, want_packet_idx=True, first_trial=7)
        monkeypatch.setenv("OFDM_FRAME_NO_LAZY", "1")
        fu, fp = e.frame_sweep(cfg, snrs, 1500, want_packet_idx=True, first_trial=7)
        monkeypatch.delenv("OFDM_FRAME_NO_LAZY")
    assert np.array_equal(lp, fp)
    assert np.array_equal(lz, fu)
    assert np.mean(lp[-4:] > 0) > 0.99


@pytest.mark.parametrize("msg_len", [96, 49, 40, 30])
def test_symbol_kernel_three_data_lanes_per_quad(pkg, monkeypatch, msg_len):
    """Messages of 3..8 data symbols run frame_sym_kernel with quads {LTF, D, D, D} (ceil(n_data / 3) quads per
    item; 12 lanes per 8-symbol item instead of 16).  Every counter and packet_idx equals the {LTF, LTF, D, D}
    layout (OFDM_FRAME_SYM_DPQ2=1), for 8-, 5-, 4- and 3-symbol messages: the item totals are summed in symbol order
    either way.  (4 symbols: the kernel derives 2 data lanes per quad from the 2-quad tile)"""
    snrs = np.array([0.0, 6.0, 10.0, 14.0, 20.0, 30.0])
    msg = (b"three data lanes per quad in the symbol kernel, one lane for the LTF estimate. " * 2)[:msg_len]
    with pkg.Engine(0) as e:
        nd = e.set_message(msg)
        assert nd == -(-8 * msg_len // 96) and nd >= 3
        cfg = pkg.make_cfg(payload="message")
        q3, p3 = e.frame_sweep(cfg, snrs, 2000, want_packet_idx=True, first_trial=5)
        monkeypatch.setenv("OFDM_FRAME_SYM_DPQ2", "1")
        q2, p2 = e.frame_sweep(cfg, snrs, 2000, want_packet_idx=True, first_trial=5)
        monkeypatch.delenv("OFDM_FRAME_SYM_DPQ2")
    assert np.array_equal(p3, p2)
    assert np.array_equal(q3, q2)
    assert q3[-1, 0] == 2000 and q3[-1, 3] == 0


def test_frame_sweep_two_chunks_equal_their_halves(engine, pkg):
    """A sweep of more than 2^22 (trial, SNR) items runs as several sync -> symbol launch pairs through the
    hand-off buffer: its counters and packet_idx equal those of two sweeps of half the trials each (one
    chunk each)."""
    cfg = pkg.make_cfg(payload="message")
    snrs = np.arange(0.0, 31.0, 2.0)
    n = 600_000                                   # 9.6M items: two chunks of at most 2^23
    whole, wp = engine.frame_sweep(cfg, snrs, n, want_packet_idx=True)
    a, ap = engine.frame_sweep(cfg, snrs, n // 2, want_packet_idx=True)
    b, bp = engine.frame_sweep(cfg, snrs, n // 2, first_trial=n // 2, want_packet_idx=True)
    assert np.array_equal(wp, np.concatenate([ap, bp], axis=1))
    assert np.array_equal(whole, a + b)


def _halved_chunk(nd, cap_items):
    """the chunk ofdm_frame_sweep ends up with (ofdm_frame.hip frame_chunk_items + the NOMEM halving loop)"""
    chunk = min(1 << 23, (1 << 23) * 3 // (1 + nd))
    while chunk > cap_items and chunk > (1 << 16):
        chunk //= 2
    return chunk


@pytest.mark.parametrize("case", ["fixed", "generic", "message8"])
def test_frame_sweep_nomem_halving_and_nonzero_q0(pkg, monkeypatch, case):
    """ADVICE r4 / VERDICT r4 Weak 8: when the hand-off buffer cannot be allocated, ofdm_frame_sweep halves its
    chunk and retries (ofdm_frame.hip, the NOMEM loop).  OFDM_DEVICE_ALLOC_CAP makes the allocation fail above a
    size, so the sweep runs in chunks whose first item is NOT a multiple of the 7-point SNR grid (q0 != 0: chunk
    item i is trial trial0 + (q0 + i) / 7, SNR (q0 + i) % 7).  Every counter and packet_idx equals the uncapped
    one-chunk sweep, for the fixed-geometry sync kernel, the generic one and an 8-symbol message."""
    snrs = np.array([0.0, 4.0, 8.0, 10.0, 12.0, 16.0, 30.0])
    nd = 8 if case == "message8" else 2
    per_item = (1 + nd) * 64 * 8 + 16                       # hand-off windows + info per item
    n = 15_000 if nd == 8 else 40_000
    if case == "generic":
        monkeypatch.setenv("OFDM_FRAME_GENERIC", "1")
    with pkg.Engine(0) as e:
        if nd == 8:
            assert e.set_message((b"halving the hand-off chunk, 8 data symbols. " * 3)[:96]) == 8
        cfg = pkg.make_cfg(payload="message")
        whole, wp = e.frame_sweep(cfg, snrs, n, want_packet_idx=True, first_trial=11)
        assert e.scratch_bytes() >= len(snrs) * n * per_item     # one chunk
        released = e.trim()
        assert released > 0 and e.scratch_bytes() == 0
        target = 65536 if nd == 2 else 43690
        cap = int(1.05 * target * per_item)
        assert _halved_chunk(nd, cap // per_item) == target
        assert len(snrs) * n > 2 * target and target % len(snrs) != 0      # >= 3 chunks, q0 != 0 from chunk 2 on
        monkeypatch.setenv("OFDM_DEVICE_ALLOC_CAP", str(cap))
        part, pp = e.frame_sweep(cfg, snrs, n, want_packet_idx=True, first_trial=11)
        assert 0 < e.scratch_bytes() <= cap + 4096
        monkeypatch.delenv("OFDM_DEVICE_ALLOC_CAP")
    assert np.array_equal(pp, wp)
    assert np.array_equal(part, whole)
    assert whole[0, 0] == n and np.mean(wp[-2:] > 0) > 0.99


def test_frame_sweep_nomem_below_the_smallest_chunk(pkg, monkeypatch):
    """a cap below the smallest chunk's buffer is an OFDM_E_NOMEM error, not a crash or a partial result"""
    with pkg.Engine(0) as e:
        monkeypatch.setenv("OFDM_DEVICE_ALLOC_CAP", str(10 << 20))
        with pytest.raises(pkg.abi.OfdmError, match="OFDM_DEVICE_ALLOC_CAP"):
            e.frame_sweep(pkg.make_cfg(payload="message"), [10.0], 100_000)
        monkeypatch.delenv("OFDM_DEVICE_ALLOC_CAP")
        c = e.frame_sweep(pkg.make_cfg(payload="message"), [30.0], 1000)      # the context is still usable
        assert c[0, 0] == 1000


def _drop_trials(sweep, snrs, trials, n_counters=16):
    """counters of the given trials (one call each, same SNR grid, so the same streams)"""
    acc = np.zeros((len(snrs), n_counters), np.int64)
    for t in trials:
        acc += sweep(int(t))
    return acc


def test_frame_sweep_evm_counters_vs_oracle(engine, oracle, pkg):
    """The counters behind Output_EVM_AGC.txt / Output_EVM_AGC_DB.txt (OFDM.c:1104-1150, 1228-1231):
    EVM_PRE_Q (7), EVM_POST_AXIS (8), EVMDB_PRE_Q (9), EVMDB_POST_Q (10), EVMDB_POST_FINITE (11) of
    the batched sweep (frame_sym_kernel<false, 2>) vs the oracle on the same Philox streams.  Trials
    whose packet_idx differs (fp32 vs double at the 0.75 threshold) are re-run one by one on both
    sides and subtracted, so the remaining trials are compared tightly."""
    snrs = [0.0, 3.0, 6.0, 8.0, 10.0, 14.0, 30.0]
    n = 400
    cfg_g, cfg_o = pkg.make_cfg(payload="message"), oracle.cfg(payload="message")
    g, gp = engine.frame_sweep(cfg_g, snrs, n, want_packet_idx=True)
    o, op = oracle.frame_sweep(cfg_o, snrs, 0, n, "c", dump_pidx=True)
    bad = np.nonzero(np.any(gp != op, axis=0))[0]
    assert len(bad) <= 0.01 * n * len(snrs), len(bad)
    g = g - _drop_trials(lambda t: engine.frame_sweep(cfg_g, snrs, 1, first_trial=t), snrs, bad)
    o = o - _drop_trials(lambda t: oracle.frame_sweep(cfg_o, snrs, t, 1, "c"), snrs, bad)
    nf = g[:, 0]
    assert np.array_equal(nf, o[:, 0]) and np.all(nf == n - len(bad))
    assert np.array_equal(g[:, 5], o[:, 5])                                   # sync failures
    q = 2.0 ** 20
    # before the slicer: per-frame sum |z - d|^2 (fp32 vs double) and per-frame EVM_dB
    assert np.all(np.abs(g[:, 7] - o[:, 7]) <= 2e-5 * o[:, 7] + nf), (g[:, 7], o[:, 7])
    assert np.all(np.abs(g[:, 9] - o[:, 9]) / q <= 1e-3 * nf), (g[:, 9] / q / nf, o[:, 9] / q / nf)
    # after the slicer: axis errors and finite-frame counts exact up to near-threshold decisions
    d8, d11 = np.abs(g[:, 8] - o[:, 8]), np.abs(g[:, 11] - o[:, 11])
    assert np.all(d8 <= 2) and np.all(d11 <= 1), (g[:, 8], o[:, 8], g[:, 11], o[:, 11])
    assert np.all(np.abs(g[:, 10] - o[:, 10]) / q <= 1e-3 * nf + 25.0 * (d8 + d11))
    # the regimes are all present: sync failures, slicer errors in every frame, none at all
    assert o[0, 5] > 0 and o[0, 11] == nf[0] and o[-1, 11] == 0 and o[-1, 8] == 0


def _curve_rows():
    return json.loads((GOLDEN / "ref_mc_curve.json").read_text())["rows"]


def _evm_batches(engine, pkg, snr, batches, per_batch):
    """per-batch mean per-trial EVM_dB before / after the slicer, and finite post-slicer counts"""
    cfg = pkg.make_cfg(payload="message")
    pre, post, fin, frames = [], [], [], []
    for b in range(batches):
        c = engine.frame_sweep(cfg, snr, per_batch, first_trial=b * per_batch)
        pre.append(c[:, 9] / 2.0 ** 20 / c[:, 0])
        post.append(c[:, 10] / 2.0 ** 20 / np.maximum(c[:, 11], 1))
        fin.append(c[:, 11]); frames.append(c[:, 0])
    return np.array(pre), np.array(post), np.sum(fin, axis=0), np.sum(frames, axis=0)


def test_reference_evm_curve(engine, pkg):
    """configs[2] "reproduce Output_EVM_AGC.txt": the mean per-trial EVM_dB of the GPU frame sweep
    vs the compiled reference's own trial loop (ref_mc_curve.json, 48000 trials/point), before the
    slicer at every point 0..30 dB and after it where the reference mean is finite (0..2 dB: every
    trial has slicer errors) or -inf (3..30 dB: some trial has none, OFDM.c:1148-1150).  Bound: 5
    standard errors of the difference (GPU batch spread, reference scaled by its trial count) plus
    0.03 dB for the RNG difference (glibc-style rand() Box-Muller vs Philox, D8)."""
    rows = _curve_rows()
    snr = np.array([r["snr_db"] for r in rows])
    K, B = 16, 25_000
    pre_b, post_b, fin, frames = _evm_batches(engine, pkg, snr, K, B)
    for i, r in enumerate(rows):
        m = pre_b[:, i].mean()
        se = pre_b[:, i].std(ddof=1) / np.sqrt(K)
        se_ref = pre_b[:, i].std(ddof=1) * np.sqrt(B / r["trials"])
        tol = 5 * np.hypot(se, se_ref) + 0.03
        print(f"{r['snr_db']:5.1f} dB  EVM pre: GPU {m:8.3f}  reference {r['mean_evm_db']:8.3f}  "
              f"diff {m - r['mean_evm_db']:+.3f}  tol {tol:.3f}")
        assert abs(m - r["mean_evm_db"]) < tol, (r["snr_db"], m, r["mean_evm_db"], tol)
        ref_post = r["mean_evm_agc_db"]
        # trials without any slicer error make the reference's mean -inf: expected count in its sample
        lam = (frames[i] - fin[i]) / frames[i] * r["trials"]
        if np.isfinite(ref_post):
            assert lam < 5, (r["snr_db"], lam)             # P(none of 48000 | lam >= 5) < 0.7 %
            mp = post_b[:, i].mean()
            sp = post_b[:, i].std(ddof=1)
            tolp = 5 * np.hypot(sp / np.sqrt(K), sp * np.sqrt(B / r["trials"])) + 0.03
            print(f"{r['snr_db']:5.1f} dB  EVM post: GPU {mp:8.3f}  reference {ref_post:8.3f}  tol {tolp:.3f}")
            assert abs(mp - ref_post) < tolp, (r["snr_db"], mp, ref_post)
        else:
            assert lam > 0.01, (r["snr_db"], lam)          # P(at least one of 48000 | lam <= 0.01) < 1 %


def test_frame_sweep_noiseless_and_edges(engine, pkg):
    cfg = pkg.make_cfg(payload="message", noise="none")
    c, p = engine.frame_sweep(cfg, [20.0], 2000, want_packet_idx=True)
    assert c[0, 3] == 0 and c[0, 5] == 0                           # no sync failure without noise
    assert np.all(p > 0)
    c0 = engine.frame_sweep(cfg, [20.0], 0)                        # empty
    assert c0[0, 0] == 0
    with pytest.raises(Exception):
        engine.frame_sweep(pkg.make_cfg(payload="random"), [10.0], 10)   # needs a fixed payload


def test_frame_sweep_capture_lengths(engine, pkg):
    """The filtered frame shares the capture's LDS region when the region has 4 nfr + 20 samples
    (1970: tight fit, 3008: default) and has its own region otherwise (1500).  With the first frame
    at capture sample 400 and the next at 1380, every length selects the same packet, and the
    waveform-indexed noise makes the frame samples identical: all counters agree."""
    cfg_n = pkg.make_cfg(payload="message", noise="none")
    cfg = pkg.make_cfg(payload="message")
    for c, snrs in ((cfg_n, [20.0]), (cfg, [16.0, 20.0])):
        res = [engine.frame_sweep(c, snrs, 64, fixed_start=580, want_packet_idx=True, cap_len=L)
               for L in (1500, 1970, 3008)]
        for cnt, pidx in res[1:]:
            assert np.array_equal(pidx, res[0][1])
            assert np.array_equal(cnt, res[0][0])
        assert np.all(res[0][1] > 0)
        if c is cfg_n:
            assert np.all(res[0][1] == res[0][1][0, 0]) and res[0][0][0, 3] == 0


def _snr_at(snr, ber, level):
    """SNR where log10(BER) crosses `level` (linear interpolation of log BER)."""
    lb = np.log10(np.maximum(ber, 1e-12))
    for i in range(len(snr) - 1):
        if lb[i] >= level > lb[i + 1]:
            return snr[i] + (lb[i] - level) / (lb[i] - lb[i + 1]) * (snr[i + 1] - snr[i])
    return None


def _gpu_ber_batches(engine, pkg, snr, batches, per_batch):
    """per-batch BER (bit errors / bits) and frame-error counts of the GPU frame sweep"""
    cfg = pkg.make_cfg(payload="message")
    ber, ferr = [], []
    for k in range(batches):
        c = engine.frame_sweep(cfg, snr, per_batch, first_trial=k * per_batch)
        ber.append(c[:, 3] / c[:, 2])
        ferr.append(c[:, 4])
    return np.array(ber), np.sum(ferr, axis=0)


@pytest.mark.slow
def test_reference_ber_curve_within_tenth_db(engine, pkg):
    """north_star: reproduce the reference BER-vs-SNR curve within +-0.1 dB, down the waterfall.

    Reference: the compiled OFDM.c's own trial loop (ref_mc_curve.json; 48000 trials/point, 1e6 at
    11, 12 dB and 4e6 at 13, 14, 15 dB where the curve is set by rare failed frames, OFDM.c:752-761, BER
    OFDM.c:1152-1161, loop OFDM.c:1195-1222).  GPU: 1e7 trials/point in 50 batches.  The SNR where log10
    BER crosses each level (log-linear interpolation between the 1-dB points) must agree within 0.1 dB at
    every level from 10^-1 down to 10^-5 (the deepest whose crossing lies inside the 15-dB fixture; its
    bracketing points 14 / 15 dB hold 2513 / 309 reference trials with errors, >= 100 required).  Point-wise, the two means agree within 5 frame-clustered standard errors: the reference's from
    its per-trial BER variance (a failed sync costs ~half the bits at once) plus a pseudo-count of one
    failed frame, the GPU's from the spread of its 50 batches."""
    rows = [r for r in json.loads((GOLDEN / "ref_mc_curve.json").read_text())["rows"] if r["snr_db"] <= 15]
    snr = np.array([r["snr_db"] for r in rows])
    ref = np.array([r["ber"] for r in rows])
    n_ref = np.array([r["trials"] for r in rows], float)
    fails = np.array([r["trials_ber_pos"] for r in rows])
    K, B = 50, 200_000
    bb, ferr = _gpu_ber_batches(engine, pkg, snr, K, B)
    ber = bb.mean(axis=0)
    se_gpu = bb.std(axis=0, ddof=1) / np.sqrt(K)
    se_ref = np.sqrt((np.array([r["ber_trial_var"] for r in rows]) * n_ref + 0.25) / n_ref ** 2)
    checked = []
    for level in np.arange(-1.0, -5.01, -0.5):
        s_ref, s_gpu = _snr_at(snr, ref, level), _snr_at(snr, ber, level)
        if s_ref is None:
            break
        i = int(np.searchsorted(snr, s_ref))            # bracketing reference points i - 1, i
        if min(fails[i - 1], fails[i]) < 100:
            break
        assert s_gpu is not None, level
        print(f"BER 1e{level:+.1f}: reference {s_ref:.3f} dB, GPU {s_gpu:.3f} dB, offset {s_gpu - s_ref:+.3f} dB "
              f"(reference failed frames {fails[i - 1]} / {fails[i]})")
        assert abs(s_ref - s_gpu) < 0.1, (level, s_ref, s_gpu)
        checked.append(level)
    assert min(checked) <= -5.0, checked                # the waterfall down to 1e-5, not just its shoulder
    for s, b, r, eg, er, fe in zip(snr, ber, ref, se_gpu, se_ref, ferr):
        z = (b - r) / np.hypot(eg, er)
        print(f"{s:5.1f} dB  BER GPU {b:.4e}  reference {r:.4e}  z {z:+.2f}  GPU frame errors {fe}")
        assert abs(z) < 5, (s, b, r, eg, er)


def test_reference_main_evm_files_vs_reference_curve(pkg, tmp_path):
    """main()'s EVM files at SNR 6..40 (OFDM.c:1195-1231) with 100k trials per point vs the reference
    curve: Output_EVM_AGC.txt (mean per-trial EVM_dB before the slicer) within the fixture's sampling
    error + the "%.2e" rounding of the file; Output_EVM_AGC_DB.txt -inf wherever the reference's
    mean is -inf (3..30 dB)."""
    from ofdm_amd import sweep
    sweep.reference_main(tmp_path, trials=100_000)
    snr = pkg.read_float_array_file(tmp_path / "Output_SNR.txt")
    pre = pkg.read_float_array_file(tmp_path / "Output_EVM_AGC.txt")
    post = pkg.read_float_array_file(tmp_path / "Output_EVM_AGC_DB.txt")
    side = json.loads((tmp_path / "ofdm_sweep.json").read_text())
    assert side["evm_files"] == "trial"
    curve = {r["snr_db"]: r for r in _curve_rows()}
    hits = 0
    for s, e, ep, exact in zip(snr, pre, post, side["mean_trial_evm_db"]):
        assert e == float("%.2e" % np.float32(exact))
        if s in curve:
            hits += 1
            r = curve[s]
            ulp = 0.5 * 10 ** (np.floor(np.log10(abs(r["mean_evm_db"]))) - 2)
            sd_trial = 10.0 if s <= 12 else 1.0      # per-trial EVM_dB spread (sync failures below 13 dB)
            tol = 5 * sd_trial * np.sqrt(1 / 100_000 + 1 / r["trials"]) + 0.03
            assert abs(e - r["mean_evm_db"]) < tol + ulp, (s, e, r["mean_evm_db"])
            assert np.isneginf(ep) and np.isneginf(r["mean_evm_agc_db"])
    assert hits == 18
    assert np.all(np.isneginf(post))


def test_reference_main_writes_files(pkg, tmp_path):
    """main() mirror: SNR 6..40, four files in the reference format (OFDM.c:1228-1231)."""
    from ofdm_amd import sweep
    res = sweep.reference_main(tmp_path, trials=200)
    files = sorted(p.name for p in tmp_path.iterdir())
    assert files == sorted(["Output_SNR.txt", "Output_EVM_AGC.txt", "Output_EVM_AGC_DB.txt", "Output_BER.txt",
                            "ofdm_sweep.json"])
    snr = pkg.read_float_array_file(tmp_path / "Output_SNR.txt")
    assert np.array_equal(snr, np.arange(6, 41))
    ber = pkg.read_float_array_file(tmp_path / "Output_BER.txt")
    assert ber[0] > 1e-3 and np.all(ber[-10:] == 0)
    evm = pkg.read_float_array_file(tmp_path / "Output_EVM_AGC.txt")
    assert evm[-1] < -35
    assert res.counters.shape == (35, 16)


def test_reference_main_evm_finite_files(pkg, tmp_path):
    """--evm finite: Output_EVM_AGC_DB.txt holds the mean post-slicer EVM_dB over the trials that have one
    (finite where any trial had a slicer error), the finite counts go to the sidecar; the pre-slicer file is
    the default's."""
    from ofdm_amd import sweep
    snr = np.arange(6.0, 13.0)
    (tmp_path / "t").mkdir()
    (tmp_path / "f").mkdir()
    res = sweep.reference_main(tmp_path / "t", trials=2000, snr_db=snr)
    sweep.reference_main(tmp_path / "f", trials=2000, snr_db=snr, evm="finite")
    pre_t = pkg.read_float_array_file(tmp_path / "t" / "Output_EVM_AGC.txt")
    pre_f = pkg.read_float_array_file(tmp_path / "f" / "Output_EVM_AGC.txt")
    post_f = pkg.read_float_array_file(tmp_path / "f" / "Output_EVM_AGC_DB.txt")
    side = json.loads((tmp_path / "f" / "ofdm_sweep.json").read_text())
    assert np.array_equal(pre_t, pre_f)
    fin = np.array(side["post_finite_trials"])
    assert np.all(fin > 0) and np.all(fin < 2000)            # some trials clean, some with slicer errors
    assert np.all(np.isfinite(post_f))
    want = res.counters[:, pkg.abi.C_EVMDB_POST_Q] / pkg.abi.EVM_Q_SCALE / fin
    assert np.allclose(post_f, [float("%.2e" % np.float32(v)) for v in want], rtol=0, atol=0.006)
