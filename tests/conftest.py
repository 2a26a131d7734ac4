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
