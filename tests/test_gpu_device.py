"""Device functions of the frame kernels checked on the GPU in isolation (test programs built in-tree by
tests/device/build_device.py with the library's hipcc flags).

atan2_cfo (ofdm_device.h) replaces atan2f in the coarse / fine CFO estimates (OFDM.c:798, 821).  ADVICE r4: its
claim to equal the device library's atan2f was covered only by sweep-level tests.  Here it is compared with
atan2f on the same GPU, bit for bit, on random arguments over 2^-140 .. 2^100, on both axes, on signed zeros and
on subnormals."""
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
EXE = ROOT / "tests" / "device" / "_build" / "atan2_check"


def _run(tmp_path, y, x):
    assert EXE.exists(), "built by __graft_entry__.build() (tests/device/build_device.py)"
    inp = np.stack([np.asarray(y, np.float32), np.asarray(x, np.float32)], axis=1)
    (tmp_path / "in.bin").write_bytes(inp.tobytes())
    r = subprocess.run([str(EXE), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), np.float32).reshape(-1, 2)
    return out[:, 0], out[:, 1]


def test_atan2_cfo_equals_device_atan2f(tmp_path):
    rng = np.random.default_rng(5)
    n = 1 << 20
    mag = np.exp2(rng.uniform(-140, 100, (2, n)))           # normal and subnormal magnitudes, wide ratios
    y = (mag[0] * rng.choice([-1, 1], n)).astype(np.float32)
    x = (mag[1] * rng.choice([-1, 1], n)).astype(np.float32)
    # CFO-like sums: comparable magnitudes, every quadrant
    z = rng.standard_normal((2, 1 << 16)).astype(np.float32)
    y = np.concatenate([y, z[0]]); x = np.concatenate([x, z[1]])
    got, lib = _run(tmp_path, y, x)
    assert np.all(np.isfinite(got))
    bad = got.view(np.uint32) != lib.view(np.uint32)
    # bit for bit wherever the result is normal; when atan2 itself underflows (|y / x| < 2^-126) the quotient is
    # subnormal and the library's frexp-scaled division may round it one subnormal step differently
    normal = np.abs(lib) >= np.finfo(np.float32).tiny
    assert not (bad & normal).any(), list(zip(y[bad & normal][:5], x[bad & normal][:5], got[bad & normal][:5]))
    assert np.all(np.abs(got[bad].astype(np.float64) - lib[bad]) <= 2 * 1.4e-45)
    assert bad.mean() < 1e-2
    np.testing.assert_allclose(got, np.arctan2(y.astype(np.float64), x.astype(np.float64)), rtol=3e-7, atol=3e-45)


def test_atan2_cfo_edges(tmp_path):
    tiny = np.float32(1e-45)                                 # the smallest subnormal
    sub = np.float32(3e-39)
    vals = np.array([0.0, -0.0, 1.0, -1.0, tiny, -tiny, sub, -sub, 2.0 ** -70, 2.0 ** 70, 3.0e38, -3.0e38], np.float32)
    y, x = np.meshgrid(vals, vals, indexing="ij")
    y = y.ravel(); x = x.ravel()
    got, lib = _run(tmp_path, y, x)
    assert np.all(np.isfinite(got)), "a NaN phase would corrupt the trial's CFO"
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    # normal results to 3e-7; results that underflow (|y / x| < 2^-126) to two subnormal steps
    under = np.abs(ref) < np.finfo(np.float32).tiny
    off = np.where(under, np.abs(got - ref) > 2.8e-45, ~np.isclose(got, ref, rtol=3e-7, atol=0))
    assert not off.any(), [(float(a), float(b), float(c), float(d), float(e))
                           for a, b, c, d, e in zip(y[off], x[off], got[off], ref[off], lib[off])]
    # signed zeros as atan2f: (+-0, +0) -> +-0, (+-0, -0) -> +-pi
    for yy, xx, want in ((0.0, 0.0, 0.0), (-0.0, 0.0, -0.0), (0.0, -0.0, np.pi), (-0.0, -0.0, -np.pi)):
        k = np.flatnonzero((y.view(np.uint32) == np.float32(yy).view(np.uint32)) &
                           (x.view(np.uint32) == np.float32(xx).view(np.uint32)))[0]
        assert got[k] == np.float32(want) and np.signbit(got[k]) == np.signbit(want), (yy, xx, got[k])
    # (m, m) -> pi/4 at every scale, the largest included (rcp(m) would underflow without the scaling)
    for m in (tiny, sub, 1.0, 3.0e38):
        k = np.flatnonzero((y == np.float32(m)) & (x == np.float32(m)))[0]
        assert got[k] == np.float32(np.pi / 4), (m, got[k])
    same = (got.view(np.uint32) == lib.view(np.uint32)) | (np.abs(lib) < np.finfo(np.float32).tiny)
    assert same.all(), (y[~same], x[~same], got[~same], lib[~same])
