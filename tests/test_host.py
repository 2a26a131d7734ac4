"""Host-side checks that need no GPU: the C-ABI library loads and exports every symbol its header
declares, the ctypes structs match the header, the file writer keeps the reference format."""
import json
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def header_functions():
    h = (ROOT / "include" / "ofdm_mi355x.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(ofdm_\w+)\(", h, re.M)))


def test_header_matches_binding(pkg):
    assert header_functions() == sorted(pkg.abi.EXPORTS)


def test_library_loads_and_exports(pkg):
    lib = pkg.load_library()      # raises if the HIP library is missing: no fallback
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.ofdm_abi_version() == pkg.abi.ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", str(pkg.abi.LIB_PATH)], capture_output=True, text=True).stdout
    for name in header_functions():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_has_gfx950_code_object(pkg):
    # the embedded HIP fat binary names its only target
    blob = pkg.abi.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_struct_layout(pkg):
    import ctypes as C
    assert C.sizeof(pkg.abi.Cfg) == 48
    assert C.sizeof(pkg.abi.RxOpts) == 32


def test_errors_without_context(pkg):
    lib = pkg.load_library()
    # a NULL context must be rejected with an error code and a message, never exit()
    rc = lib.ofdm_fft64(None, None, None, 0, 0, 0)
    assert rc == -1 and b"bad" in lib.ofdm_last_error()
    rc = lib.ofdm_tx_bytes(-1, None, None)
    assert rc == -1


def test_tx_bytes(pkg):
    import ctypes as C
    lib = pkg.load_library()
    tb, bb = C.c_int64(), C.c_int64()
    assert lib.ofdm_tx_bytes(17, C.byref(tb), C.byref(bb)) == 0
    # 17 frames = 34 symbols -> pitch = 64 (whole wave) + 64 (guard wave); rows of 80 samples x 8 B
    assert tb.value == 80 * 128 * 8 and bb.value == 3 * 128 * 4
    assert lib.ofdm_tx_bytes(1 << 23, C.byref(tb), C.byref(bb)) == 0
    assert lib.ofdm_tx_bytes((1 << 23) + 1, C.byref(tb), C.byref(bb)) == -1     # int32 element offsets


def test_write_float_array_format(pkg, tmp_path):
    p = tmp_path / "x.txt"
    pkg.write_float_array_to_file([6, -10.84, float("-inf"), 0.0, 3.5e-5], p)
    assert p.read_text() == "6.00e+00\t-1.08e+01\t-inf\t0.00e+00\t3.50e-05\n"
    assert np.allclose(pkg.read_float_array_file(p)[[0, 1, 3, 4]], [6, -10.8, 0, 3.5e-5])


def test_reference_files_parse(pkg, tmp_path):
    files = json.loads((GOLDEN / "reference_data.json").read_text())
    for name, text in files.items():
        (tmp_path / name).write_text(text)
        v = pkg.read_float_array_file(tmp_path / name)
        assert len(v) == 35
    snr = pkg.read_float_array_file(tmp_path / "Output_SNR.txt")
    assert np.array_equal(snr, np.arange(6, 41))


def test_write_reference_outputs_refuses_missing_dir(pkg, tmp_path):
    with pytest.raises(FileNotFoundError):
        pkg.write_reference_outputs(tmp_path / "nope", [1], [1], [1], [1])


@pytest.mark.skipif(not (ROOT.parent / "reference" / "scripts" / "OFDM_Plotting.py").exists(),
                    reason="reference scripts only exist in the build container")
def test_reference_plotting_script_reads_our_files(pkg, tmp_path):
    """scripts/OFDM_Plotting.py must drop in unchanged.  It resolves data/ and results/ relative to
    its own location, so it is run from a scratch copy of its directory layout."""
    pytest.importorskip("matplotlib")
    import shutil
    base = tmp_path / "ref"
    (base / "scripts").mkdir(parents=True)
    (base / "data").mkdir()
    shutil.copy(ROOT.parent / "reference" / "scripts" / "OFDM_Plotting.py", base / "scripts")
    snr = np.arange(6, 41)
    pkg.write_reference_outputs(base / "data", snr, -snr - 1.3, np.full(35, -np.inf), np.where(snr < 10, 1e-2, 0))
    r = subprocess.run([sys.executable, str(base / "scripts" / "OFDM_Plotting.py")], capture_output=True, text=True,
                       env={"MPLBACKEND": "Agg", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stderr
    assert "Extracted 35 valid numbers" in r.stdout
    assert (base / "results" / "ber_vs_snr.png").exists()


def test_shard_ranges(pkg):
    from ofdm_amd import dist
    for n in (0, 1, 7, 1000, 10 ** 7 + 3):
        for w in (1, 2, 3, 8):
            rs = [dist.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
