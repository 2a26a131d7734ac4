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
def test_pipelined_step_equals_symbol_sweep(engine, pkg):
    import torch
    b = _bench()
    cfg = pkg.make_cfg(est="ls", noise="real", channel="awgn", conv="c", payload="random")
    first, frames = 1000, b.PIPE_CHUNKS * b.MIN_PIPE_FRAMES + 77
    chunks = b.plan_chunks(first, frames)
    assert len(chunks) == b.PIPE_CHUNKS
    counters = engine.new_counters(len(b.SNR_GRID))
    step = b.PipelinedSymbolStep(torch, engine, cfg, chunks, counters, 0)
    for _ in range(2):                    # twice: the second step reuses both batches
        step()
    torch.cuda.synchronize()
    got = counters.cpu().numpy()
    want = engine.symbol_sweep(cfg, b.SNR_GRID, frames, first_frame=first)
    assert np.array_equal(got, want)
