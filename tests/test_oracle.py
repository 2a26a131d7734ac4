"""Pin the CPU restatement (oracle/ofdm_oracle.c) to the reference's own outputs.

Golden data (tests/golden/, made by tests/golden/gen_golden.py from the compiled, unmodified
/root/reference/src/OFDM.c and from data/Matlab_Output.txt) -- these tests run without the
reference tree."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, load_golden, normwise


def test_philox_known_answers(oracle):
    # Random123 kat_vectors for philox4x32_10
    assert [int(v) for v in oracle.philox([0, 0, 0, 0], [0, 0])] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert [int(v) for v in oracle.philox([0xffffffff] * 4, [0xffffffff] * 2)] == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert [int(v) for v in oracle.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                                          [0xa4093822, 0x299f31d0])] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_gauss_moments(oracle):
    z = np.concatenate([oracle.gauss4([i, 0, 7, 0x5A000000], [0x80211A, 0]) for i in range(20000)])
    assert abs(z.mean()) < 0.02 and abs(z.var() - 1) < 0.03


def test_fft_vectors_vs_reference(oracle):
    g = load_golden("fft_vectors.npz")
    for x, f, i in zip(g["x"], g["fft"], g["ifft"]):
        # reference fp32 with double twiddles vs exact: ~1e-7 normwise
        assert normwise(f, oracle.fft64(x.astype(np.complex128))) < 1e-6
        assert normwise(i, oracle.ifft64(x.astype(np.complex128), "c")) < 1e-6


def test_ifft_convention_shift(oracle):
    # C ifft = MATLAB ifft circularly shifted by 32 samples (D5)
    rng = np.random.default_rng(1)
    X = rng.standard_normal(64) + 1j * rng.standard_normal(64)
    assert np.allclose(oracle.ifft64(X, "c"), np.roll(oracle.ifft64(X, "matlab"), 32), atol=1e-12)


def test_tx_waveform_vs_reference(oracle):
    g = load_golden("tx_waveform.npz")
    bits = oracle.message_bits(b"Hey! I am Vivaswan")
    assert np.array_equal(bits, g["bits"])
    assert np.allclose(oracle.rrc_taps(True), g["rrc_taps"], atol=0, rtol=0)
    w = oracle.frame_waveform(bits, "c", True, 10)
    assert normwise(w, g["waveform"]) < 1e-6
    _, _, lf = oracle.preambles("c")
    assert np.array_equal(lf, g["ltf_freq"])
    # Data_Payload_Mod (OFDM.c:515-517)
    mod = np.concatenate([oracle.data_symbol(bits[96 * d:96 * d + 96])[16:] for d in range(2)])
    X = np.concatenate([np.fft.fftshift(np.fft.fft(mod[64 * d:64 * d + 64] * (-1) ** np.arange(64)))
                        for d in range(2)])
    assert mod.shape == (128,) and np.isfinite(X).all()
    # P_tx / P_sym = 0.4980
    P = np.mean(np.abs(g["waveform"].astype(np.complex128)) ** 2)
    assert abs(P / (52 / 4096) - 0.4980) < 5e-4


def test_receiver_stages_vs_reference(oracle):
    """Injected-noise captures through Receiver() (compiled reference) vs the restatement."""
    g = load_golden("rx_stages.npz")
    tw = load_golden("tx_waveform.npz")
    w = tw["waveform"].astype(np.complex128)
    bits = tw["bits"]
    for k in range(len(g["snr"])):
        rs = int(g["rx_start"][k])
        cap = w[rs:rs + 3008] + g["noise"][k].astype(np.float64)
        o = oracle.receiver_frame(cap, bits, "c", dumps=True)
        assert o["packet_idx"] == int(g["packet_idx"][k])
        assert normwise(o["corr"], g["corr"][k]) < 1e-5
        assert normwise(o["rxframe"], g["rxframe"][k]) < 1e-5
        assert normwise(o["fine"], g["fine"][k]) < 1e-4
        assert normwise(o["H"], g["H"][k]) < 1e-4
        ref_np = g["nopilot"][k]
        assert normwise(o["nopilot"], ref_np) < 1e-4
        # decisions identical except for components within 1e-4 of the slicer threshold
        near = (np.abs(ref_np.real) < 1e-4) | (np.abs(ref_np.imag) < 1e-4)
        diff = (o["bits"] != g["bits"][k]).reshape(-1, 2).any(axis=1)
        assert not np.any(diff & ~near)
        np.testing.assert_allclose(o["res"][0], g["res"][k][0], atol=2e-3)
        assert o["res"][2] == pytest.approx(float(g["res"][k][2]), abs=1e-6)


def test_matlab_known_answer(oracle):
    """data/Matlab_Output.txt: noiseless MATLAB Tester, capture [0,3000), RX_Payload_1_demod (D6)."""
    kat = load_golden("matlab_output.npz")["bits"]
    tb = oracle.tester_bits()
    assert np.sum(kat != tb[:96]) == 3          # the KAT carries 3 bit errors by construction
    w = oracle.frame_waveform(tb, "matlab", False, 10)
    o = oracle.receiver_frame(w[:3000], tb, "matlab")
    assert np.array_equal(o["bits"][:96], kat)


def test_c_receiver_with_tester_payload(oracle):
    # OFDM.c cannot reproduce the KAT; with the Tester payload it makes 13/192 errors
    tb = oracle.tester_bits()
    w = oracle.frame_waveform(tb, "c", True, 10)
    o = oracle.receiver_frame(w[:3008], tb, "c")
    assert int(np.sum(o["bits"] != tb)) == 13 and int(np.sum(o["bits"][:96] != tb[:96])) == 11


def test_frame_mode_mc_matches_reference_curve(oracle):
    """Oracle frame-mode Monte Carlo vs the reference's own trial loop (ref_mc_curve.json)."""
    curve = {r["snr_db"]: r for r in json.loads((GOLDEN / "ref_mc_curve.json").read_text())["rows"]}
    snrs = [6.0, 8.0, 12.0]
    cnt = oracle.frame_sweep(oracle.cfg(payload="message"), snrs, 0, 600, "c")
    for s, c in zip(snrs, cnt):
        ber = c[3] / c[2]
        ref = curve[s]["ber"]
        # frame-clustered errors: sd of mean per-trial BER ~ 0.25/sqrt(n) at these SNRs
        sd = 0.5 * np.sqrt(ref * (1 - ref) / 600) + 0.25 / np.sqrt(600) * (ref > 0.01) + 1e-3
        assert abs(ber - ref) < 5 * sd, (s, ber, ref)


def test_symbol_mode_theory(oracle):
    """Ideal-CSI AWGN symbol chain vs closed form: BER = 1.5p - p^2 (non-Gray map, D10),
    p = Q(sqrt(64 snr / (52 kappa)))."""
    from math import erfc, sqrt
    cfg = oracle.cfg(est="ideal")
    snrs = [0.0, 3.0]
    cnt = oracle.symbol_sweep(cfg, snrs, 0, 3000)
    for s, c in zip(snrs, cnt):
        snr = 10 ** (s / 10)
        p = 0.5 * erfc(sqrt(64 * snr / (52 * 0.4980)) / sqrt(2))
        theory = 1.5 * p - p * p
        ber = c[3] / c[2]
        assert abs(ber - theory) < 5 * sqrt(theory / c[2]) * 2, (s, ber, theory)


def test_symbol_ls_pair_noise_matches_reference_estimator(oracle):
    """Symbol-mode LS forms H from FFT(r1 + r2) with the pair noise drawn once as sqrt(2) x N(0, s^2)
    (DESIGN.md §3).  Against the reference's own Channel_Estimation on two separately noised LTF
    windows (tests/golden/ref_genie_ls_curve.json, 20k frames/point): same BER and pre-slicer EVM."""
    import json
    from math import sqrt
    rows = json.loads((GOLDEN / "ref_genie_ls_curve.json").read_text())["rows"]
    snrs = [r["snr_db"] for r in rows]
    cnt = oracle.symbol_sweep(oracle.cfg(), snrs, 0, 6000)
    for r, c in zip(rows, cnt):
        p_ref, p = r["bit_err"] / r["bits"], c[3] / c[2]
        sd = sqrt(3 * p_ref / r["bits"] + 3 * p / c[2])          # 2 correlated bits per QPSK symbol
        assert abs(p - p_ref) < 5 * sd, (r["snr_db"], p, p_ref)
        # pooled ZF EVM is heavy-tailed below ~4 dB (|H| near 0 outliers): compare where it converges
        if r["snr_db"] >= 4:
            evm_ref = 10 * np.log10(r["sum_evm_pre"] / r["evm_terms"])
            evm = 10 * np.log10(c[7] / 2 ** 20 / c[6])
            assert abs(evm - evm_ref) < 0.05, (r["snr_db"], evm, evm_ref)


def _chain_rows():
    return {r["snr_db"]: r for r in json.loads((GOLDEN / "ref_symbol_chain_curve.json").read_text())["rows"]}


def test_symbol_chain_fixture_reproduces(reflib):
    """tests/golden/ref_symbol_chain_curve.json is what gen_golden.py --only chain writes: its 30 dB row
    regenerated here job by job (the reference's stage functions, ref_time_symbol_chain) is identical."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    import gen_golden
    res = [(snr, reflib.symbol_chain_stats(snr, n, seed).tolist()) for snr, n, seed in gen_golden.chain_jobs([30.0])]
    assert gen_golden.chain_rows(res) == [_chain_rows()[30.0]]


def test_oracle_evm_matches_reference_chain_to_30db(oracle):
    """Pre-slicer EVM of the oracle's LS symbol chain vs the reference's stage-function chain
    (ref_symbol_chain_curve.json) from 8 to 30 dB: EVM ~ -(SNR + 2.2) dB, within 0.05 dB."""
    rows = _chain_rows()
    snrs = [8.0, 14.0, 20.0, 30.0]
    cnt = oracle.symbol_sweep(oracle.cfg(), snrs, 0, 4000)
    for s, c in zip(snrs, cnt):
        evm_ref = 10 * np.log10(rows[s]["sum_evm_pre"] / rows[s]["evm_terms"])
        evm = 10 * np.log10(c[7] / 2 ** 20 / c[6])
        assert abs(evm - evm_ref) < 0.05, (s, evm, evm_ref)
