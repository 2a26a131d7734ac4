"""Shared fixtures.  `-m "not gpu"` tests run anywhere (oracle vs golden fixtures, ABI exports,
host logic, gloo multi-process); `-m gpu` tests need an MI355X and call the HIP library through
the C ABI, comparing against the oracle (tests/ is one of the oracle's permitted users)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(ROOT))

import ofdm_pkg  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running statistical test")


@pytest.fixture(scope="session")
def pkg():
    return ofdm_pkg.load()


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle, build_oracle  # noqa: PLC0415
    build_oracle()
    return Oracle()


@pytest.fixture(scope="session")
def reflib():
    from oracle import RefLib, REF_SO  # noqa: PLC0415
    if not REF_SO.exists():
        pytest.skip("oracle/_ref not built (needs the reference source)")
    return RefLib()


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def engine(pkg):
    eng = pkg.Engine(0)
    yield eng
    eng.close()


def normwise(a, b) -> float:
    a = np.asarray(a); b = np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def off_threshold_pidx_mismatches(engine, oracle, wave, snrs, gp, op, cap_len, seed=0x80211A, first_trial=0):
    """The frame-sweep trials whose packet_idx differs between the GPU (gp) and the oracle (op) although the
    decision is NOT on Packet_Selection's 0.75 threshold.  A trial's capture is rebuilt from the sweep's own
    streams (Transmission_Over_Air of `wave`, capture start from the Philox start stream, OFDM.c:949); the
    reference's selection (tests/test_lazy_rule.packet_selection, pinned to the compiled reference) is re-run with
    the threshold moved by up to +-0.1 %.  A mismatch is explained when that moves the decision and one of the two
    packet_idx is among the decisions reached: fp32 sliding sums (GPU) against double ones (oracle) at M ~ 0.75."""
    from test_lazy_rule import corr_out, packet_selection  # noqa: PLC0415
    bad = []
    for q, t in np.argwhere(gp != op):
        q, tr = int(q), first_trial + int(t)
        rs = int(oracle.philox([tr, 0, 0, 0x5B000000 | q], [seed, 0])[0] % (len(wave) - cap_len))
        ota = engine.transmission_over_air(wave, snrs[q], seed=seed, trial=tr, snr_index=q)
        m = corr_out(ota[rs:rs + cap_len].astype(np.complex128))
        moved = {packet_selection(m, 0.75 * (1 + d)) for d in np.linspace(-1e-3, 1e-3, 21)}
        if not (len(moved) > 1 and {int(gp[q, t]), int(op[q, t])} & moved):
            bad.append((q, tr, int(gp[q, t]), int(op[q, t]), sorted(moved)))
    return bad
