"""bench.py's step plan (CPU) and its pipelined symbol step against one ofdm_symbol_sweep (GPU): the
benchmark's own code path must produce the counters a plain sweep produces."""
import importlib.util
import json
import sys

import numpy as np
import pytest

from conftest import ROOT


def _bench():
    """bench.py as the module `bench` (one instance: its cpu_baseline workers are pickled by reference)"""
    if "bench" not in sys.modules:
        spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
        mod = importlib.util.module_from_spec(spec)
        sys.modules["bench"] = mod
        spec.loader.exec_module(mod)
    return sys.modules["bench"]


@pytest.mark.parametrize("first,frames", [(0, 0), (0, 7), (5, 1_000_000), (0, 1 << 20), (123, 5_000_000),
                                          (0, 50_000_000), (0, (1 << 23) * 3 + 5)])
def test_plan_chunks(first, frames):
    b = _bench()
    ch = b.plan_chunks(first, frames)
    assert sum(n for _, n in ch) == frames
    pos = first
    for a, n in ch:                       # contiguous, in order, non-empty, at most one batch each
        assert a == pos and 0 < n <= b.MAX_CHUNK_FRAMES
        pos += n
    if frames:
        sizes = [n for _, n in ch]
        assert max(sizes) - min(sizes) <= 1
    if frames >= b.PIPE_CHUNKS * b.MIN_PIPE_FRAMES:
        assert len(ch) >= b.PIPE_CHUNKS   # the Tx pipeline has chunks to overlap
    elif frames:
        assert len(ch) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("channel", ["awgn", "rayleigh4"])
def test_pipelined_step_equals_symbol_sweep(engine, pkg, fused, channel):
    import torch
    b = _bench()
    cfg = pkg.make_cfg(est="ls", noise="real", channel=channel, conv="c", payload="random")
    first, frames = 1000, b.PIPE_CHUNKS * b.MIN_PIPE_FRAMES + 77
    chunks = b.plan_chunks(first, frames)
    assert len(chunks) == b.PIPE_CHUNKS
    counters = engine.new_counters(len(b.SNR_GRID))
    step = b.PipelinedSymbolStep(torch, engine, cfg, chunks, counters, 0, fused=fused)
    for _ in range(2):                    # twice: the second step reuses both batches
        step()
    torch.cuda.synchronize()
    got = counters.cpu().numpy()
    want = engine.symbol_sweep(cfg, b.SNR_GRID, frames, first_frame=first)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(conv="c", payload="random"), dict(conv="matlab", payload="message"),
                                dict(conv="c", payload="tester", channel="rayleigh4"),
                                dict(conv="c", payload="random", noise="complex"),     # not fused: Tx launch
                                dict(conv="c", payload="random", est="ideal")])        # not fused: Tx launch
def test_fused_next_tx_equals_tx_kernel(engine, pkg, kw):
    """ofdm_set_next_tx: the batch the packed LS receiver builds in its group prologues is byte-identical to
    the Tx kernel's, for batches with more and with fewer groups than the receiver's launch (ragged sizes),
    and the receiver's own counters are unchanged by the extra work.  Receivers that do not fuse it launch
    the Tx kernel first: same bytes."""
    import torch
    cfg = pkg.make_cfg(**{"est": "ls", "noise": "real", **kw})
    snr = [0.0, 10.0]
    tx0, bits0 = engine.tx_frames(cfg, 5, 1000)
    want_cnt = engine.rx_frames(cfg, tx0, bits0, 5, 1000, snr).cpu().numpy()
    for f1, n1 in ((1005, 2001), (3006, 333), (7, 64)):       # 2001 frames: the loop over groups gg + G
        tx_ref, bits_ref = engine.tx_frames(cfg, f1, n1)
        tx, bits = engine.tx_buffers(n1)
        tx.fill_(-1.0)
        bits.fill_(-1)
        engine.set_next_tx(cfg, f1, n1, tx, bits)
        cnt = engine.rx_frames(cfg, tx0, bits0, 5, 1000, snr)
        torch.cuda.synchronize()
        assert np.array_equal(cnt.cpu().numpy(), want_cnt)
        n_sym = (2 * n1 + 63) // 64 * 64
        a = tx_ref.view(torch.uint8).cpu().numpy().reshape(80, -1)
        g = tx.view(torch.uint8).cpu().numpy().reshape(80, -1)
        assert np.array_equal(a[:, :8 * n_sym], g[:, :8 * n_sym]), (f1, n1)
        a = bits_ref.cpu().numpy().reshape(10, -1)
        g = bits.cpu().numpy().reshape(10, -1)
        assert np.array_equal(a[:, :n_sym], g[:, :n_sym]), (f1, n1)


def _fake_pmc(build_id, kernel="rx_pack_kernel"):
    return {"kernels": [kernel], "valu_instr_per_unit": 52.6, "hbm_bytes_per_unit": 90.0, "build_id": build_id,
            "issue_model": {"cap_frac": 0.585, "waves_per_simd": 2, "build_id": build_id}}


def test_roofline_needs_pmc_of_the_loaded_build(pkg):
    """bench.py reports a VALU roofline fraction only from a PMC record stamped with the build id of the
    library it loaded (codeobj: hash of the kernel's gfx950 code + descriptor); a mutated or missing id,
    or a record of another kernel, gives frac null with the reason."""
    from ofdm_amd import abi, codeobj
    b = _bench()
    lib_id = codeobj.workload_build_id(abi.library_file(), "c3")
    assert lib_id and len(lib_id) == 16
    assert codeobj.workload_build_id(abi.library_file(), "c4") == lib_id          # same receiver instance
    assert len({codeobj.workload_build_id(abi.library_file(), w) for w in ("c2", "c3", "c5", "frame")}) == 4
    args = ("rx_pack_kernel", "c3", 4e7, 3.4e-3, 16, True)
    ok, traffic = b.make_roofline(_fake_pmc(lib_id), lib_id, *args)
    assert ok["frac"] == pytest.approx(4e7 * 52.6 / 3.4e-3 / b.VALU_PEAK_PER_S)
    assert ok["pmc_build_id"] == ok["lib_build_id"] == lib_id and traffic == 90.0 * 4e7
    assert ok["issue_model_cap_frac"] == 0.585 and "profiled_clock_ghz" not in ok
    # with the SQ clock of the certified PMC run, the same fractions at that clock (clock vs issue efficiency)
    clocked = {**_fake_pmc(lib_id), "clock_ghz": 2.2}
    ck, _ = b.make_roofline(clocked, lib_id, *args)
    assert ck["frac"] == ok["frac"] and ck["profiled_clock_ghz"] == 2.2
    assert ck["frac_at_profiled_clock"] == pytest.approx(ok["frac"] * 2.4 / 2.2)
    assert ck["frac_of_issue_model_cap_at_profiled_clock"] == pytest.approx(ok["frac"] / 0.585 * 2.4 / 2.2)
    mutated = lib_id[:-1] + ("0" if lib_id[-1] != "0" else "1")
    for pmc, why in ((_fake_pmc(mutated), "stale"), (_fake_pmc(None), "stale"), ({}, "no PMC"),
                     (_fake_pmc(lib_id, "rx_ls_kernel"), "launches")):
        r, traffic = b.make_roofline(pmc, lib_id, *args)
        assert r["frac"] is None and r["achieved"] is None and traffic is None
        assert why in r["frac_null_reason"], r["frac_null_reason"]
        assert "issue_model_cap_frac" not in r
    # an issue-model record of another build is dropped, the PMC count of this build kept
    pmc = _fake_pmc(lib_id)
    pmc["issue_model"]["build_id"] = mutated
    r, _ = b.make_roofline(pmc, lib_id, *args)
    assert r["frac"] is not None and "issue_model_cap_frac" not in r


def test_dynamic_mix_cap(tmp_path):
    """tools/mix_cap.py prices the measured class counters (ambiguous classes once slow, once fast) and
    bench.py reports the run's fraction of both ends of that range."""
    sys.path.insert(0, str(ROOT / "tools"))
    import mix_cap
    from isa_mix import COST
    c = {"SQ_INSTS_VALU": 100.0, "SQ_INSTS_VALU_FMA_F32": 50.0, "SQ_INSTS_VALU_TRANS_F32": 10.0,
         "SQ_INSTS_VALU_INT64": 10.0}
    lo, hi, shares = mix_cap.price(c, 3)
    k = COST[3]
    assert lo == pytest.approx(200 / (50 * k["fast"] + 10 * k["trans"] + 40 * k["slow"]))
    assert hi == pytest.approx(200 / (80 * k["fast"] + 10 * k["trans"] + 10 * k["slow"]))
    assert shares["ambiguous"] == pytest.approx(0.3) and lo < hi
    rows = [{"Kernel_Name": "ofdm::frame_sync_kernel(ofdm::FrameArgs)", "Counter_Name": n, "Counter_Value": str(v)}
            for n, v in c.items()]
    d = tmp_path / "pass"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w") as f:
        f.write("Kernel_Name,Counter_Name,Counter_Value\n")
        f.writelines(f"\"{r['Kernel_Name']}\",{r['Counter_Name']},{r['Counter_Value']}\n" for r in rows)
    assert mix_cap.counters([d, d], mix_cap.SETS["frame"])["SQ_INSTS_VALU"] == 100.0   # counted once
    b = _bench()
    cap = b.issue_cap({"issue_model": {"method": "dynamic", "cap_frac": lo, "cap_frac_range": [lo, hi],
                                       "waves_per_simd": 3}}, 0.5)
    assert cap["frac_of_issue_model_cap_range"] == pytest.approx([0.5 / hi, 0.5 / lo])
    # the point estimate with frame's classified split of the ambiguous instructions (cndmask priced as such)
    mix = {"sync": {"classes_per_item": {"fast": 60.0, "slow": 30.0, "trans": 10.0, "cnd": 2.0},
                    "class_check_per_item": {k: {"model": v} for k, v in
                                             (("fma_f32", 40.0), ("mul_f32", 5.0), ("add_f32", 5.0),
                                              ("int64", 15.0), ("cvt", 5.0))}}}
    split = mix_cap.frame_split(mix)
    assert split == pytest.approx({"fast": 10 / 22, "slow": 10 / 22, "cnd": 2 / 22})
    est = mix_cap.price_split(c, 3, split)
    assert est == pytest.approx(200 / (k["fast"] * (50 + 30 * 10 / 22) + 10 * k["trans"] +
                                       k["slow"] * (10 + 30 * 10 / 22) + k["cnd"] * 30 * 2 / 22))
    assert est < hi
    cap = b.issue_cap({"issue_model": {"method": "dynamic_split", "cap_frac": est, "cap_frac_range": [lo, hi],
                                       "waves_per_simd": 3, "split_source": "x"}}, 0.5)
    assert cap["issue_model_cap_frac"] == est and cap["frac_of_issue_model_cap"] == pytest.approx(0.5 / est)


def test_classified_frame_cap(tmp_path):
    """tools/frame_mix.py finds the sync kernel's phases in the current gfx950 assembly (round-0 capture passes,
    the per-run offsets, the blocks round 0's decision skips), recovers the undecided fraction from a VALU count
    made with it, and bench.py reports one cap number for the classified record."""
    sys.path.insert(0, str(ROOT / "tools"))
    import frame_mix
    sync_text, sym_text = frame_mix.asm("ofdm_frame_fix.hip"), frame_mix.asm("ofdm_frame_sym.hip")
    sbb = frame_mix.kernel_blocks(sync_text, frame_mix.SYNC)
    w = frame_mix.weights(sbb, 2.0)
    assert sum(1 for a, b in w.values() if b) >= 5                # the undecided path spans several blocks
    assert any(0 < a < 1 for a, b in w.values())                  # the per-run offsets
    cls, _, _ = frame_mix.tally(sbb, w)
    items, u = 1000.0, 0.4
    d = tmp_path / "pass"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w") as f:
        f.write("Kernel_Name,Counter_Name,Counter_Value\n")
        f.write(f"\"ofdm::frame_sync_kernel<2, 3008, 4>(ofdm::FrameArgs)\",SQ_INSTS_VALU,"
                f"{items * (cls['valu'][0] + u * cls['valu'][1])}\n")
        f.write(f"\"ofdm::frame_sym_kernel<false, 2>(ofdm::FrameArgs)\",SQ_INSTS_VALU,{items * 130}\n")
    m = frame_mix.model([d], items, 3, sync_text, sym_text)
    assert m["undecided_fraction"] == pytest.approx(u)
    assert 0.5 < m["sync"]["cap_frac"] < 0.9 and 0.5 < m["cap_frac"] < 0.9
    cap = _bench().issue_cap({"issue_model": {"method": "classified", "cap_frac": m["cap_frac"], "waves_per_simd": 3,
                                              "undecided_fraction": u}}, 0.5)
    assert cap["issue_model_cap_frac"] == m["cap_frac"] and "issue_model_cap_frac_range" not in cap


def test_kernel_build_id_tracks_code_bytes(pkg, tmp_path):
    """The id is a hash of the kernel's machine code: flipping one byte of it in a copy of the library
    changes the id of that workload and no other's."""
    from ofdm_amd import abi, codeobj
    lib = abi.library_file()
    syms = codeobj.kernel_symbols(lib)
    name = next(n for n in syms if "rx_pack_kernelILi2ELi0ELi0ELb0E" in n and not n.endswith(".kd"))
    blob = bytearray(lib.read_bytes())
    at = blob.find(syms[name])
    assert at > 0
    blob[at + 100] ^= 0xFF
    mod = tmp_path / "lib_mutated.so"
    mod.write_bytes(bytes(blob))
    assert codeobj.workload_build_id(mod, "c3") != codeobj.workload_build_id(lib, "c3")
    assert codeobj.workload_build_id(mod, "c5") == codeobj.workload_build_id(lib, "c5")


def test_kernel_build_id_ignores_code_placement(pkg, tmp_path):
    """The descriptor's code-entry offset (bytes 16-23 of the .kd) moves when another kernel of the library
    changes size: the id ignores it, while any other descriptor byte (register / LDS settings) counts."""
    from ofdm_amd import abi, codeobj
    lib = abi.library_file()
    syms = codeobj.kernel_symbols(lib)
    kd = next(n for n in syms if "rx_pack_kernelILi2ELi0ELi0ELb0E" in n and n.endswith(".kd"))
    blob = bytes(lib.read_bytes())
    at = blob.find(syms[kd])
    assert at > 0 and blob.count(syms[kd]) == 1
    for off, same in ((17, True), (20, True), (0, False), (48, False)):
        b = bytearray(blob)
        b[at + off] ^= 0x01
        mod = tmp_path / f"lib_kd_{off}.so"
        mod.write_bytes(bytes(b))
        assert (codeobj.workload_build_id(mod, "c3") == codeobj.workload_build_id(lib, "c3")) == same, off


def test_kernel_build_id_covers_non_inlined_callees(pkg, monkeypatch):
    """a device function the compiler did not inline is code the kernel runs.  The id hashes every
    non-kernel function of the code object that holds the kernel, and nothing of the other code objects."""
    from ofdm_amd import codeobj
    FUNC, OBJ = codeobj.STT_FUNC, 1

    def objs(callee: bytes, other: bytes):
        return [{"k_frame_sync_kernelILi2ELi3008E": (FUNC, b"\x01" * 8), "k_frame_sync_kernelILi2ELi3008E.kd":
                 (OBJ, bytes(64)), "helper_fn": (FUNC, callee), "__hip_cuid_x": (OBJ, b"\x00")},
                {"rx_pack_kernelILi2ELi0ELi0ELb0E": (FUNC, b"\x02" * 8), "other_fn": (FUNC, other)}]
    ids = {}
    for key, args in (("a", (b"\xaa", b"\x00")), ("callee", (b"\xab", b"\x00")), ("other", (b"\xaa", b"\x01"))):
        monkeypatch.setattr(codeobj, "_code_objects", lambda p, m, _a=args: objs(*_a))
        ids[key] = codeobj.kernel_build_id(__file__, ("frame_sync_kernelILi2ELi3008E",))
    assert ids["a"] != ids["callee"] and ids["a"] == ids["other"]


def test_host_cpu_share_is_derived(monkeypatch):
    b = _bench()
    monkeypatch.setattr(b, "_cgroup_cpu_quota", lambda: (3.0, "cgroup v2 cpu.max 300000/100000"))
    s = b.host_cpu_share()
    assert s["cores"] == min(3, s["affinity"]) and "cpu.max" in s["source"]
    monkeypatch.setattr(b, "_cgroup_cpu_quota", lambda: (None, "no cgroup CPU quota"))
    assert b.host_cpu_share()["cores"] == b.host_cpu_share()["affinity"]


@pytest.mark.parametrize("workload", ["c3", "c2"])
def test_torchrun_rank0_times_the_reference(reflib, monkeypatch, workload):
    """Under torchrun (WORLD_SIZE=2) rank 0's line carries cpu_baseline with the derived core count; the
    other rank does not time it.  c2 times the ideal-CSI chain (no per-SNR Channel_Estimation)."""
    import argparse
    b = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    assert b.wants_cpu_baseline(argparse.Namespace(no_cpu_baseline=False))
    share = {"cores": 2, "affinity": 8, "quota": 2.0, "source": "cgroup v2 cpu.max 200000/100000", "visible": 8}
    cpu = b.cpu_baseline(workload, seconds=0.3, share=share)
    assert cpu["kind"] == "reference" and cpu["cores"] == 2 and cpu["value"] > 0
    assert "cpu.max" in cpu["cores_source"] and cpu["single_core"]["cores"] == 1
    assert ("known channel" in cpu["sample"]) == (workload == "c2")
    monkeypatch.setenv("RANK", "1")
    assert not b.wants_cpu_baseline(argparse.Namespace(no_cpu_baseline=False))


def test_ideal_chain_skips_the_estimate(reflib):
    """ref_time_symbol_chain with the known channel: at high SNR both chains are error-free; at 0 dB the LS
    estimate's noise costs BER (the ideal chain's is lower), and the ideal chain is faster per frame."""
    snr = np.array([0.0, 30.0])
    t_ls, a_ls = reflib.time_symbol_chain(snr, 400, seed=5)
    t_id, a_id = reflib.time_symbol_chain(snr, 400, seed=5, ideal=True)
    assert a_id[1] == a_ls[1] == 400 * 2 * 96 * 2
    assert a_id[0] < a_ls[0]


@pytest.mark.gpu
def test_pending_next_tx_survives_a_failed_rx_and_is_built_by_symbol_sweep(engine, pkg):
    """ofdm_set_next_tx + an rx call that fails its argument checks: the batch stays pending (nothing
    written), and the next valid rx call builds it.  ofdm_symbol_sweep builds a pending batch before its own
    work.  Either way the bytes are the Tx kernel's."""
    import ctypes as C
    import torch
    cfg = pkg.make_cfg(est="ls", noise="real", conv="c", payload="random")
    tx0, bits0 = engine.tx_frames(cfg, 0, 256)
    tx_ref, bits_ref = engine.tx_frames(cfg, 4096, 300)
    torch.cuda.synchronize()

    def fresh():
        tx, bits = engine.tx_buffers(300)
        tx.fill_(-1.0)
        bits.fill_(-1)
        torch.cuda.synchronize()
        return tx, bits

    def same(tx, bits):
        torch.cuda.synchronize()
        n = (2 * 300 + 63) // 64 * 64
        a = tx_ref.view(torch.uint8).cpu().numpy().reshape(80, -1)[:, :8 * n]
        g = tx.view(torch.uint8).cpu().numpy().reshape(80, -1)[:, :8 * n]
        return np.array_equal(a, g) and np.array_equal(bits_ref.cpu().numpy().reshape(10, -1)[:, :n],
                                                       bits.cpu().numpy().reshape(10, -1)[:, :n])

    tx, bits = fresh()
    engine.set_next_tx(cfg, 4096, 300, tx, bits)
    cnt = engine.new_counters(2)
    snr = np.array([0.0, 10.0])
    eq = torch.zeros(8, device="cuda:0")
    rc = engine.lib.ofdm_rx_frames_dump(engine.ctx, C.byref(cfg), C.c_void_p(tx0.data_ptr()),
                                        C.c_void_p(bits0.data_ptr()), 0, 256, snr.ctypes.data_as(C.c_void_p), 2,
                                        C.c_void_p(cnt.data_ptr()), C.c_void_p(eq.data_ptr()), None)
    assert rc == -1                                      # OFDM_E_ARG: dump with d_eq only
    torch.cuda.synchronize()
    assert np.all(bits.cpu().numpy() == -1)              # the pending batch was not consumed
    engine.rx_frames(cfg, tx0, bits0, 0, 256, snr, cnt)  # the next valid call builds it
    assert same(tx, bits)

    tx, bits = fresh()
    engine.set_next_tx(cfg, 4096, 300, tx, bits)
    engine.symbol_sweep(cfg, [5.0], 1000)                # flushes the pending batch first
    assert same(tx, bits)

    # a pending batch that shares bytes with the call's own batch is refused (it would be written
    # while read, or by two groups of one launch), and stays pending
    tx, bits = fresh()
    engine.set_next_tx(cfg, 4096, 300, tx, bits)
    sub_bits = bits[64:]                                  # overlaps the pending batch's bit rows
    rc = engine.lib.ofdm_txrx_frames(engine.ctx, C.byref(cfg), 0, 20, C.c_void_p(tx0.data_ptr()),
                                     C.c_void_p(sub_bits.data_ptr()), snr.ctypes.data_as(C.c_void_p), 2,
                                     C.c_void_p(cnt.data_ptr()))
    assert rc == -1 and b"overlaps" in engine.lib.ofdm_last_error()
    rc = engine.lib.ofdm_rx_frames(engine.ctx, C.byref(cfg), C.c_void_p(tx.data_ptr()), C.c_void_p(bits0.data_ptr()),
                                   0, 256, snr.ctypes.data_as(C.c_void_p), 2, C.c_void_p(cnt.data_ptr()))
    assert rc == -1                                      # reading the batch that is to be built
    torch.cuda.synchronize()
    assert np.all(bits.cpu().numpy() == -1)
    engine.rx_frames(cfg, tx0, bits0, 0, 256, snr, cnt)
    assert same(tx, bits)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(conv="c", payload="random"), dict(conv="matlab", payload="message"),
                                dict(conv="c", payload="tester", channel="rayleigh4"),
                                dict(conv="c", payload="random", est="ideal"),
                                dict(conv="matlab", payload="random", est="ideal"),
                                dict(conv="c", payload="random", noise="complex")])    # not packed: Tx launch
def test_txrx_equals_tx_then_rx(engine, pkg, kw):
    """ofdm_txrx_frames: the packed receivers build each group's own symbols in the group prologue and read
    them back in the same launch.  The batch is byte-identical to the Tx kernel's and the counters equal
    ofdm_rx_frames on that batch, for ragged sizes (tail groups split over blocks build their group more than
    once), more groups than the grid has blocks (a block builds its next item's group in the prologue of the
    item before), more SNR points than one launch holds (later launches read the batch the first one built),
    and with a pending ofdm_set_next_tx batch built in the same launch."""
    import torch
    cfg = pkg.make_cfg(**{"est": "ls", "noise": "real", **kw})
    for first, n, snr in ((5, 1000, [0.0, 10.0]), (3006, 333, list(np.arange(0.0, 40.0, 2.0))), (7, 64, [4.0]),
                          (11, 40_000, [2.0, 8.0]), (13, 120_000, [2.0, 8.0, 14.0])):
        tx_ref, bits_ref = engine.tx_frames(cfg, first, n)
        want = engine.rx_frames(cfg, tx_ref, bits_ref, first, n, snr).cpu().numpy()
        tx, bits = engine.tx_buffers(n)
        tx.fill_(-1.0)
        bits.fill_(-1)
        nx_ref, nxb_ref = engine.tx_frames(cfg, first + n, 700)
        nx, nxb = engine.tx_buffers(700)
        nx.fill_(-1.0)
        nxb.fill_(-1)
        engine.set_next_tx(cfg, first + n, 700, nx, nxb)
        _, _, cnt = engine.txrx_frames(cfg, first, n, snr, tx, bits)
        torch.cuda.synchronize()
        assert np.array_equal(cnt.cpu().numpy(), want), (kw, first, n)
        for (a, b), nf in (((tx_ref, tx), n), ((nx_ref, nx), 700)):
            n_sym = (2 * nf + 63) // 64 * 64
            ga = a.view(torch.uint8).cpu().numpy().reshape(80, -1)[:, :8 * n_sym]
            gb = b.view(torch.uint8).cpu().numpy().reshape(80, -1)[:, :8 * n_sym]
            assert np.array_equal(ga, gb), (kw, first, n, nf)
        for (a, b), nf in (((bits_ref, bits), n), ((nxb_ref, nxb), 700)):
            n_sym = (2 * nf + 63) // 64 * 64
            assert np.array_equal(a.cpu().numpy().reshape(10, -1)[:, :n_sym], b.cpu().numpy().reshape(10, -1)[:, :n_sym])


@pytest.mark.gpu
def test_pipelined_ideal_step_equals_symbol_sweep(engine, pkg):
    """c2's step (ideal CSI, fused Tx: one txrx launch per chunk 0) against one ofdm_symbol_sweep"""
    import torch
    b = _bench()
    cfg = pkg.make_cfg(est="ideal", noise="real", channel="awgn", conv="c", payload="random")
    for first, frames in ((1000, b.PIPE_CHUNKS * b.MIN_PIPE_FRAMES + 77), (3, 500_000)):
        chunks = b.plan_chunks(first, frames)
        counters = engine.new_counters(len(b.SNR_GRID))
        step = b.PipelinedSymbolStep(torch, engine, cfg, chunks, counters, 0, fused=True)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        want = engine.symbol_sweep(cfg, b.SNR_GRID, frames, first_frame=first)
        assert np.array_equal(counters.cpu().numpy(), want)


def test_trace_frac_keeps_the_timed_launches(tmp_path):
    """tools/trace_frac.py: from a rocprofv3 kernel trace of the bench command, the receiver dispatches of the
    timed steps only (warm-up first, in dispatch order), summed per bench launch, priced as bench.make_roofline."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("trace_frac", ROOT / "tools" / "trace_frac.py")
    tf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tf)
    d = tmp_path / "trace"
    d.mkdir()
    rows = ["Kind,Dispatch_Id,Kernel_Name,Start_Timestamp,End_Timestamp"]
    t, did = 0, 0
    # 2 warm-up + 3 timed steps of a frame-like launch: 2 chunks x (sync, sym) per step, one bench launch per step
    for step in range(5):
        for chunk in range(2):
            for k, dur in (("ofdm::frame_sync_kernel<2, 3008, 4>(ofdm::FrameArgs)", 900 if step < 2 else 1000),
                           ("void ofdm::frame_sym_kernel<false, 2>(ofdm::FrameArgs)", 100)):
                did += 1
                rows.append(f'KERNEL_DISPATCH,{did},"{k}",{t},{t + dur}')
                t += dur + 10
            did += 1
            rows.append(f'KERNEL_DISPATCH,{did},"__amd_rocclr_fillBufferAligned",{t},{t + 5}')
    (d / "run_kernel_trace.csv").write_text("\n".join(rows) + "\n")
    line = {"steps": 3, "warmup": 2, "roofline": {"kernel": "frame_sync_kernel+frame_sym_kernel", "launches": 3,
                                                  "units_per_launch": 1e6, "instr_per_unit": 10.0, "peak": 1e12,
                                                  "frac": 0.0045, "avg_launch_ms": 0.0022}}
    b = tmp_path / "line.json"
    b.write_text(json.dumps(line) + "\n")
    rec, per = tf.split(tf.receiver_dispatches(d, "frame_sync_kernel+frame_sym_kernel"), line)
    assert per == 4 and len(rec) == 12
    ns = tf.launch_ns(rec, per)
    assert ns == [2200, 2200, 2200]                       # the warm-up's 900-ns sync dispatches are dropped
    out = tmp_path / "frac.json"
    tf.main([str(d), str(b), "--out", str(out)])
    r = json.loads(out.read_text())
    assert r["trace_frac"] == pytest.approx(1e6 * 10.0 / 2.2e-6 / 1e12)
    # the line's own HIP-event mean launch time (2.2 us here) prices the same: no difference
    assert r["line_events_frac"] == pytest.approx(r["trace_frac"]) and abs(r["frac_rel_diff"]) < 1e-9


def test_c2_breakdown(tmp_path):
    """tools/c2_breakdown.py: clock from GRBM_GUI_ACTIVE over the timed receiver dispatches, the SNR loop's share
    of time (stamps, wave 0) and of VALU (issue model), and the loop's own fraction = line x 2.4 / clock x VALU
    share / time share."""
    sys.path.insert(0, str(ROOT / "tools"))
    import c2_breakdown
    d = tmp_path / "clock"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp\n")
        f.write("1,\"ofdm::rx_pack_kernel<0>\",GRBM_GUI_ACTIVE,8000000,0,1000000\n")        # warm-up: 1 GHz
        for k in range(2, 5):                                                             # timed: 2 GHz
            f.write(f"{k},\"ofdm::rx_pack_kernel<0>\",GRBM_GUI_ACTIVE,16000000,0,1000000\n")
    assert c2_breakdown.clock_ghz(d, 1) == pytest.approx(2.0)
    st = tmp_path / "stamps.txt"
    st.write_text("pack stamp wave 0: item-top barrier 5.00%; prologue work 20.00%; SNR loop 75.00%;\n"
                  "pack stamp wave 2: item-top barrier 1.00%; prologue work 9.00%; SNR loop 90.00%;\n")
    assert c2_breakdown.stamps(st) == {"item-top barrier": 0.05, "prologue work": 0.2, "SNR loop": 0.75}


def test_child_command_runs_n_ranks_of_the_same_bench():
    """`bench.py --gpus N` outside torchrun starts N ranks under torch.distributed.run as a child
    (127.0.0.1 rendezvous), with the same bench arguments, so every rank sees WORLD_SIZE == --gpus."""
    b = _bench()
    argv = ["--gpus", "4", "--workload", "c4", "--steps", "3"]
    cmd = b.child_command(4, argv, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29555" in cmd
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == argv


@pytest.mark.parametrize("world,gpus", [("3", "2"), ("1", "8"), ("2", "1")])
def test_world_size_must_equal_gpus(world, gpus):
    """Under torchrun a rank whose WORLD_SIZE differs from --gpus exits non-zero before anything is timed or
    touches the GPU (no line can carry n_gpus != --gpus)."""
    import os
    import subprocess
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE=world)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", gpus, "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert r.returncode != 0 and f"WORLD_SIZE={world} but --gpus {gpus}" in r.stderr
    assert r.stdout.strip() == ""


def test_launch_ranks_relays_one_line(monkeypatch, capsys):
    """launch_ranks passes the child's other output to stderr, relays exactly one JSON line on stdout, and
    returns non-zero when the child fails or no line (or more than one) comes back."""
    b = _bench()
    line = json.dumps({"metric": "m", "value": 1.0, "n_gpus": 2})
    for script, rc_want, out_want in ((f"print('progress'); print({line!r})", 0, line),
                                      (f"print({line!r}); raise SystemExit(3)", 3, ""),
                                      ("print('no line')", 1, ""),
                                      (f"print({line!r}); print({line!r})", 1, "")):
        monkeypatch.setattr(b, "child_command", lambda n, argv, port, _s=script: [sys.executable, "-c", _s])
        rc = b.launch_ranks(2, [])
        out = capsys.readouterr()
        assert rc == rc_want and out.out.strip() == out_want, script
        if rc_want == 0:
            assert "progress" in out.err


def test_pmc_trace_fallback_matches_stats(tmp_path):
    """tools/pmc_summary.read_trace sums the kernel-trace rows where a record has no --stats summary;
    on a record that has both (round 4's certified c3 PMC run) the two agree exactly."""
    import shutil
    sys.path.insert(0, str(ROOT / "tools"))
    import pmc_summary
    src = ROOT / "profiles" / "r04" / "pmc" / "c3"
    a = pmc_summary.read_trace(src)
    dst = tmp_path / "c3"
    shutil.copytree(src / "pmc_trace", dst / "pmc_trace")
    for f in dst.glob("pmc_trace/**/*kernel_stats.csv"):
        f.unlink()
    b = pmc_summary.read_trace(dst)
    assert a and a.keys() == b.keys()
    for k in a:
        assert a[k]["calls"] == b[k]["calls"] and a[k]["total_ns"] == pytest.approx(b[k]["total_ns"])


def test_frame8_classified_cap():
    """tools/frame8_mix.py classifies frame_sync_long_kernel's own assembly (instructions attributed
    to kernel statements through the -g build's DWARF inlining records) and weights it per item.  On the committed
    round-6 PMC record the undecided fraction it fits from the FMA count agrees with the CPU simulation of the kernel's
    rules (tests/golden/frame8_path_rates.json), and the cap lies between the all-slow and all-fast pricing."""
    sys.path.insert(0, str(ROOT / "tools"))
    import frame8_mix
    d = ROOT / "profiles" / "r06" / "pmc" / "frame8"
    m = frame8_mix.model([d / "pmc_7", d / "pmc_2"], 32_000_000 / 8)          # 12-wave blocks: 3 waves on every SIMD
    assert abs(m["undecided_fraction"] - m["undecided_fraction_simulated"]) < 0.05
    assert abs(m["g_build_instr_delta"]) < 16
    assert 0.58 < m["sync"]["cap_frac"] < 0.71 and 0.55 < m["cap_frac"] < 0.75
    assert abs(m["sync"]["class_check_per_item"]["mul_f32"]["model"] /
               m["sync"]["class_check_per_item"]["mul_f32"]["measured"] - 1) < 0.1
