"""bench.py's step plan (CPU) and its pipelined symbol step against one ofdm_symbol_sweep (GPU): the
benchmark's own code path must produce the counters a plain sweep produces."""
import importlib.util

import numpy as np
import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


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
