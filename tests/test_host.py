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


def test_product_kernels_do_not_spill(pkg):
    # build_lib writes hipcc's resource-usage remarks next to the objects and refuses a spilling build;
    # this re-reads that report so a stale library built before the check cannot slip through
    from ofdm_amd import build_lib
    if not build_lib.RESOURCE_REPORT.exists():
        pytest.skip("library not built in this tree (no resource report)")
    rows = json.loads(build_lib.RESOURCE_REPORT.read_text())
    names = {x["name"] for x in rows}
    for k in ("ofdm::rx_pack_kernel<0, 0, 0, false>", "ofdm::rx_pack_kernel<2, 0, 0, false>",
              "ofdm::rx_pack_kernel<2, 0, 1, false>", "ofdm::frame_sync_kernel<2, 3008, 12>", "ofdm::frame_sync_kernel<0, 0, 4>",
              "ofdm::frame_sync_kernel<0, 0, 1>", "ofdm::frame_sym_kernel<false, 2>",
              "ofdm::frame_sym_kernel<false, 0>",
              "ofdm::rx_ls_kernel<1, 1, false>", "ofdm::tx_symbols_kernel<0>"):
        assert k in names, k
    assert build_lib.spilling_kernels(rows) == []


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


def test_every_entry_point_rejects_a_null_context(pkg):
    """Each entry point that takes an ofdm_ctx returns OFDM_E_ARG with a message for a NULL context (all
    other arguments zero / NULL), before any HIP call: an error code, never a crash or exit()."""
    import ctypes as C
    from ofdm_amd import abi
    lib = pkg.load_library()
    checked = 0
    for name, (_, argtypes) in abi._SIGS.items():
        if not argtypes or argtypes[0] is not abi._V or name == "ofdm_ctx_destroy":   # destroy(NULL) is a no-op
            continue
        args = [None if t in (abi._V, C.c_char_p) or t.__name__.startswith("LP_") else 0 for t in argtypes]
        rc = getattr(lib, name)(*args)
        assert rc == -1, (name, rc)
        assert lib.ofdm_last_error(), name
        checked += 1
    assert checked == len([n for n, (_, t) in abi._SIGS.items() if t and t[0] is abi._V]) - 1, checked
    assert lib.ofdm_ctx_destroy(None) == 0


def test_tx_bytes(pkg):
    import ctypes as C
    lib = pkg.load_library()
    tb, bb = C.c_int64(), C.c_int64()
    assert lib.ofdm_tx_bytes(17, C.byref(tb), C.byref(bb)) == 0
    # 17 frames = 34 symbols -> pitch = 64 (whole wave) + 64 (guard wave); rows of 80 samples x 8 B
    assert tb.value == 80 * 128 * 8 and bb.value == 10 * 128 * 4    # 3 payload + 4 demap + 3 pair-order words
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


REF_SCRIPTS = ROOT.parent / "reference" / "scripts"
GPU_KAT_FILE = GOLDEN / "gpu_kat_Code_Output.txt"


def _run_compare_double(cwd, code_output_text):
    """scripts/compare_double.py unchanged, as its __main__ runs it: Code_Output.txt against
    Matlab_Output.txt in the current directory with tolerance 1e-6 (compare_double.py:41-42)."""
    import shutil
    cwd.mkdir(parents=True, exist_ok=True)
    shutil.copy(REF_SCRIPTS / "compare_double.py", cwd)
    shutil.copy(ROOT.parent / "reference" / "data" / "Matlab_Output.txt", cwd)
    (cwd / "Code_Output.txt").write_text(code_output_text)
    r = subprocess.run([sys.executable, "compare_double.py"], cwd=cwd, capture_output=True, text=True,
                       env={"PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stderr
    return r.stdout


def _assert_compare_double_clean(out):
    assert out.count("Extracted 96 numbers.") == 2, out          # equal lengths: no early return
    assert "Files have different lengths" not in out
    assert "Max Error: 0.000000e+00" in out, out
    assert "Average Error: 0.000000e+00" in out, out
    assert "Mismatch" not in out, out


@pytest.mark.skipif(not (REF_SCRIPTS / "compare_double.py").exists(),
                    reason="reference scripts only exist in the build container")
def test_reference_compare_double_reads_our_code_output(pkg, oracle, tmp_path):
    """north_star: scripts/compare_*.py drop in unchanged.  The KAT receiver's bits (frame mode, MATLAB
    convention, Tester payload, noiseless capture [0, 3000): D6) written by fileio.write_bits_file are
    diffed by the unmodified compare_double.py against data/Matlab_Output.txt: zero mismatches.
    (a) bits of the oracle's KAT receiver (equal to the GPU's: tests/test_gpu_frame.py::test_matlab_known_answer);
    (b) the Code_Output.txt the GPU KAT test wrote on an MI355X (tests/golden/gpu_kat_Code_Output.txt)."""
    from ofdm_amd import fileio
    tb = oracle.tester_bits()
    w = oracle.frame_waveform(tb, "matlab", False, 10)
    o = oracle.receiver_frame(w[:3000], tb, "matlab")
    p = tmp_path / "bits.txt"
    fileio.write_bits_file(o["bits"][:96], p)
    _assert_compare_double_clean(_run_compare_double(tmp_path / "a", p.read_text()))
    assert GPU_KAT_FILE.exists(), "the GPU KAT record is committed with the tests"
    _assert_compare_double_clean(_run_compare_double(tmp_path / "b", GPU_KAT_FILE.read_text()))
    # the check is not vacuous: one flipped bit is reported as a mismatch
    bad = p.read_text().split("\t")
    bad[5] = str(1 - int(bad[5]))
    out = _run_compare_double(tmp_path / "c", "\t".join(bad))
    assert "Mismatch at index 5" in out and "Max Error: 1.000000e+00" in out


def test_shard_ranges(pkg):
    from ofdm_amd import dist
    for n in (0, 1, 7, 1000, 10 ** 7 + 3):
        for w in (1, 2, 3, 8):
            rs = [dist.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


def test_allreduce_refuses_world_without_group(pkg, monkeypatch):
    """a sharded sweep must never be written from one rank's share: with WORLD_SIZE > 1
    and no process group the reduction raises instead of silently returning."""
    import torch
    from ofdm_amd import dist as odist
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(odist.DistError):
        odist.allreduce_counters(torch.zeros((2, 16), dtype=torch.int64))
    with pytest.raises(odist.DistError):
        odist.allreduce_counters_np(np.zeros((2, 16), np.int64))
    monkeypatch.setenv("WORLD_SIZE", "1")
    c = np.arange(32, dtype=np.int64).reshape(2, 16)
    assert odist.allreduce_counters_np(c) is c


def test_mean_trial_evm_semantics(pkg):
    """Output_EVM_AGC*.txt values for trials > 1: mean of the per-trial EVM_dB; the post-slicer mean
    is -inf once any trial had no slicer error (that trial's own value is -inf, OFDM.c:1148-1150)."""
    from ofdm_amd import abi
    c = np.zeros((2, 16), np.int64)
    c[:, abi.C_FRAMES] = 4
    c[:, abi.C_EVMDB_PRE_Q] = [-40 << 20, 8 << 20]
    c[:, abi.C_EVMDB_POST_Q] = [0, 6 << 20]
    c[:, abi.C_EVMDB_POST_FINITE] = [0, 4]
    r = pkg.SweepResult(np.array([30.0, 0.0]), c)
    assert list(r.mean_frame_evm_db) == [-10.0, 2.0]
    assert np.isneginf(r.mean_frame_evm_post_db[0]) and r.mean_frame_evm_post_db[1] == 1.5
    # --evm finite: the post-slicer mean over the finite trials only (-inf only with none finite)
    c[0, abi.C_EVMDB_POST_Q], c[0, abi.C_EVMDB_POST_FINITE] = -30 << 20, 2
    r = pkg.SweepResult(np.array([30.0, 0.0]), c)
    assert np.isneginf(r.mean_frame_evm_post_db[0])
    assert list(r.mean_finite_frame_evm_post_db) == [-15.0, 1.5]
    c[0, abi.C_EVMDB_POST_FINITE] = 0
    assert np.isneginf(pkg.SweepResult(np.array([30.0, 0.0]), c).mean_finite_frame_evm_post_db[0])


def test_reference_symbol_chain_baseline_is_the_genie_workload(reflib):
    """bench.py's cpu_baseline for c2-c5 runs the reference's own stage functions as the genie symbol
    chain (ref_harness.c ref_time_symbol_chain): its BER at 0 / 4 dB is the genie fixture's."""
    rows = {r["snr_db"]: r for r in json.loads((GOLDEN / "ref_genie_ls_curve.json").read_text())["rows"]}
    for snr, n in ((0.0, 3000), (4.0, 6000)):
        t, acc = reflib.time_symbol_chain([snr], n)
        ber, ref = acc[0] / acc[1], rows[snr]["bit_err"] / rows[snr]["bits"]
        sd = np.sqrt(ref / acc[1] + ref / rows[snr]["bits"]) * 3      # ~3 bit errors per error event
        assert abs(ber - ref) < 5 * sd, (snr, ber, ref)
        assert t > 0
