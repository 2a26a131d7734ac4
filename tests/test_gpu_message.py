"""Message mode: a MESSAGE payload of any length up to 96 characters is
framed as ceil(8 len / 96) data symbols (Data_Generator, OFDM.c:435-465), transmitted, received
and decoded back to text (Message_Generator, OFDM.c:910-939, 1167-1182).  GPU vs the oracle's
restatement of Transmitter()/Receiver() for the same frame count."""
import numpy as np
import pytest

from conftest import normwise

pytestmark = pytest.mark.gpu

MSG = b"IEEE 802.11a on MI355X: a longer message, five symbols!"     # 55 chars -> 5 data symbols


@pytest.fixture
def msg_engine(pkg):
    """A separate context, so the session engine keeps the reference message."""
    eng = pkg.Engine(0)
    yield eng
    eng.close()


@pytest.fixture
def msg_oracle(oracle):
    oracle.set_message(MSG)
    yield oracle
    oracle.set_message(b"Hey! I am Vivaswan")


def test_frames_and_padding(msg_engine, oracle, pkg):
    assert msg_engine.payload_frames("message") == 2                  # OFDM.c:20 default, ceil(144 / 96)
    assert msg_engine.set_message(MSG) == 5
    assert msg_engine.payload_frames("tester") == 2
    for n, d in ((1, 1), (12, 1), (13, 2), (96, 8)):
        assert msg_engine.set_message(b"x" * n) == d
    with pytest.raises(Exception):
        msg_engine.set_message(b"x" * 97)                              # > 8 data symbols per frame
    bits = oracle.message_bits(MSG)
    assert len(bits) == 5 * 96
    assert pkg.decode_message(bits) == MSG.decode() + " " * (60 - len(MSG))   # padded with ' '


def test_transmitter_vs_oracle(msg_engine, oracle, pkg):
    from ofdm_amd import abi
    msg_engine.set_message(MSG)
    w = msg_engine.transmitter("c", "message")
    assert len(w) == abi.wave_len(5) == 14600
    ref = oracle.frame_waveform(oracle.message_bits(MSG), "c", True, 10)
    assert normwise(w, ref) < 2e-6


def test_noiseless_decode(msg_engine, pkg):
    from ofdm_amd import abi
    msg_engine.set_message(MSG)
    w = msg_engine.transmitter("c", "message")
    L = abi.capture_len(5)
    for rs in (0, 700, 4321, len(w) - L):
        o = msg_engine.receiver(w[rs:rs + L], "c", "message")
        assert o["frames"] == 5 and not o["sync_fail"]
        assert o["message"].rstrip(" ") == MSG.decode(), (rs, o["message"])


def test_receiver_vs_oracle_injected_noise(msg_engine, msg_oracle, pkg):
    from ofdm_amd import abi
    msg_engine.set_message(MSG)
    w = msg_engine.transmitter("c", "message")
    L = abi.capture_len(5)
    bits = msg_oracle.message_bits(MSG)
    P = float(np.mean(np.abs(w.astype(np.complex128)) ** 2))
    rng = np.random.default_rng(5)
    for snr, rs in ((30.0, 100), (14.0, 2500), (10.0, 6000), (8.0, 900)):
        cap = w[rs:rs + L].astype(np.complex128)
        cap.real += np.sqrt(P / 10 ** (snr / 10)) * rng.standard_normal(L)
        cap = cap.astype(np.complex64)
        g = msg_engine.receiver(cap, "c", "message")
        o = msg_oracle.receiver_frame(cap, bits, "c")
        assert g["packet_idx"] == o["packet_idx"], snr
        near = np.abs(g["eq"].real) < 1e-3
        near = np.repeat(near | (np.abs(g["eq"].imag) < 1e-3), 2)
        assert not np.any((g["bits"] != o["bits"]) & ~near), snr
        assert g["res"][0] == pytest.approx(o["res"][0], abs=2e-3)


def test_frame_sweep_vs_oracle(msg_engine, msg_oracle, pkg):
    msg_engine.set_message(MSG)
    cfg = pkg.make_cfg(payload="message")
    snrs = [8.0, 12.0]
    n = 200
    g, gp = msg_engine.frame_sweep(cfg, snrs, n, want_packet_idx=True)
    o, op = msg_oracle.frame_sweep(msg_oracle.cfg(payload="message"), snrs, 0, n, "c", dump_pidx=True)
    assert np.mean(gp == op) > 0.99
    from conftest import off_threshold_pidx_mismatches  # noqa: PLC0415
    from ofdm_amd import abi  # noqa: PLC0415
    w = msg_engine.transmitter("c", "message")
    nd = -(-8 * len(MSG) // 96)
    assert off_threshold_pidx_mismatches(msg_engine, msg_oracle, w, snrs, gp, op, abi.capture_len(nd)) == []
    for k in (0, 1, 2, 6):                                            # frames, symbols, bits, evm terms
        assert np.array_equal(g[:, k], o[:, k])
    assert g[0, 1] == 5 * n and g[0, 2] == 480 * n
    assert np.all(np.abs(g[:, 3] - o[:, 3]) <= 480 * np.sum(gp != op, axis=1) + 3)


# ---------------------------------------------------------------- word-length report (§8(f) rank 4)
def test_word_length_report_vs_oracle(engine, oracle):
    """Word_Optimization_Analysis (OFDM.c:38-73) of the RRC-filtered capture, on the reference's own
    injected-noise captures (tests/golden/rx_stages.npz)."""
    from conftest import load_golden
    g = load_golden("rx_stages.npz")
    w = load_golden("tx_waveform.npz")["waveform"]
    for k in range(len(g["snr"])):
        rs = int(g["rx_start"][k])
        cap = (w[rs:rs + 3008] + g["noise"][k]).astype(np.complex64)
        r = engine.word_length_report(cap)
        mn, mx, ma, bits = oracle.word_length(cap.astype(np.complex128))
        assert r["min"] == pytest.approx(mn, abs=1e-6) and r["max"] == pytest.approx(mx, abs=1e-6)
        assert r["max_abs"] == pytest.approx(ma, abs=1e-6)
        assert r["bits"] == bits


def test_frame_sweep_word_stats(engine, oracle, pkg):
    """The sweep's per-SNR extremes equal the extremes of the per-trial reports of the same captures."""
    from ofdm_amd import abi
    cfg = pkg.make_cfg(payload="message")
    snrs = [6.0, 20.0]
    n = 24
    c = engine.frame_sweep(cfg, snrs, n, word_stats=True)
    c0 = engine.frame_sweep(cfg, snrs, n)
    assert np.array_equal(c[:, :13], c0[:, :13])                    # opt-in stat leaves the rest alone
    w = engine.transmitter("c", "message")
    for q, s in enumerate(snrs):
        lo, hi = np.inf, -np.inf
        for t in range(n):
            rs = int(oracle.philox([t, 0, 0, 0x5B000000 | q], [0x80211A, 0])[0] % (len(w) - 3008))
            ota = engine.transmission_over_air(w, s, seed=0x80211A, trial=t, snr_index=q)
            r = engine.word_length_report(ota[rs:rs + 3008])
            lo, hi = min(lo, r["min"]), max(hi, r["max"])
        assert c[q, abi.C_WL_MIN_Q] / 2 ** 20 == pytest.approx(lo, abs=1e-5)
        assert c[q, abi.C_WL_MAX_Q] / 2 ** 20 == pytest.approx(hi, abs=1e-5)
        ma = max(abs(lo), abs(hi))
        assert c[q, abi.C_WL_BITS] == (1 if ma < 1 else int(np.ceil(np.log2(ma))) + 1)


@pytest.mark.parametrize("msg", [b"Twelve chars", b"x" * 20 + b" three syms", bytes(range(32, 127)) + b"!"],
                         ids=["1-symbol", "3-symbol", "8-symbol"])
def test_frame_sweep_vs_oracle_lengths(msg_engine, oracle, pkg, msg):
    """Frame lengths at the edges of the symbol kernel's tiling and the sync kernel's LDS budget: 1 data
    symbol (one quad per trial, an idle data lane), 3 (two quads, the second half empty) and 8 (the
    longest capture, 5955 samples: detection chunks of 47 positions, two crossing words per lane)."""
    from ofdm_amd import abi
    nd = msg_engine.set_message(msg)
    assert nd == -(-8 * len(msg) // 96)
    oracle.set_message(msg)
    try:
        w = msg_engine.transmitter("c", "message")
        L = abi.capture_len(nd)
        o = msg_engine.receiver(w[333:333 + L], "c", "message")
        assert not o["sync_fail"] and o["message"].rstrip(" ") == msg.decode()
        cfg = pkg.make_cfg(payload="message")
        snrs = [8.0, 14.0]
        n = 160
        g, gp = msg_engine.frame_sweep(cfg, snrs, n, want_packet_idx=True)
        r, rp = oracle.frame_sweep(oracle.cfg(payload="message"), snrs, 0, n, "c", dump_pidx=True)
        assert np.mean(gp == rp) > 0.99
        from conftest import off_threshold_pidx_mismatches  # noqa: PLC0415
        assert off_threshold_pidx_mismatches(msg_engine, oracle, w, snrs, gp, rp, L) == []
        for k in (0, 1, 2, 6):                                         # frames, symbols, bits, evm terms
            assert np.array_equal(g[:, k], r[:, k])
        assert g[0, 1] == nd * n and g[0, 2] == 96 * nd * n
        assert np.all(np.abs(g[:, 3] - r[:, 3]) <= 96 * nd * np.sum(gp != rp, axis=1) + 3)
    finally:
        oracle.set_message(b"Hey! I am Vivaswan")
