"""SURVEY §5 sanitizers, the fast part of tools/sanitize.py in the CPU suite: the ASan + UBSan +
LSan builds of the oracle and of the reference harness (oracle/Makefile `asan`) run their drivers
(oracle/asan_drive.c), and every report must be one of the reference's own known defects (tools/sanitize.KNOWN:
the S_k[53] over-read of OFDM.c:381, Channel_Estimation's per-call leak, OFDM.c:836-841).  Our restatement must be
clean.  The full sweep (the oracle tests on instrumented libraries, the product library's host code) is
tools/sanitize.py; its record is profiles/r06/sanitizers/."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT / "tools"))
import sanitize  # noqa: E402


@pytest.fixture(scope="module")
def asan_build():
    r = subprocess.run(["make", "-s", "asan"], cwd=ROOT / "oracle", capture_output=True, text=True)
    if r.returncode != 0:
        if not Path(os.environ.get("OFDM_REF_SRC", "/root/reference/src/OFDM.c")).exists():
            pytest.skip("the reference tree is not here (the _ref drivers need it)")
        raise AssertionError(r.stderr[-3000:])
    return ROOT / "oracle" / "_asan"


def _run(exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    return r.returncode, r.stdout + r.stderr


def test_oracle_is_sanitizer_clean(asan_build):
    rc, text = _run(asan_build / "drive_oracle")
    assert rc == 0 and "drive_oracle done" in text, text[-3000:]
    assert sanitize.classify(text) == [], text[-3000:]


def test_reference_reports_are_its_known_defects(asan_build):
    rc, text = _run(asan_build / "drive_ref")
    assert "drive_ref done" in text, text[-3000:]
    reps = sanitize.classify(text)
    assert [r for r in reps if sanitize.explain(r) is None] == [], reps
    kinds = {(r["kind"], r["where"]) for r in reps}
    assert ("stack-buffer-overflow", "Slice_Repeater <- Preamble_Generator OFDM.c:381") in kinds
    assert ("leak", "Channel_Estimation") in kinds
