"""frame_sync_long_kernel's capture ring (ofdm_frame.hip, OFDM_FRAME_LONG_TU), its index arithmetic restated on the CPU:
every float a detection round or a matched-filter run reads must be the capture sample it means, for every capture
offset, packet position and lazy outcome.  A ring slot here holds the sample index last written to it (the kernel
writes whole Philox blocks of 4 samples at float 4 (b - b0) mod LW_RING, and blocks landing in [0, LW_EXT) also at
their mirror past LW_RING).  The matched-filter window's generation draws its blocks in trimmed passes, restated at the
end."""
import numpy as np
import pytest

LW_CHUNK, LW_ROUND = 31, 64 * 31
LW_PIECE = LW_ROUND + 47
LW_RING, LW_EXT = 2976, 96
MF_RUN = 5


def red(x):
    """the kernel's two unsigned reductions: x mod LW_RING for 0 <= x < 3 LW_RING"""
    m = 0xFFFFFFFF
    x &= m
    x = min(x, (x - LW_RING) & m)
    return min(x, (x - LW_RING) & m)


class Ring:
    def __init__(self, rx_start):
        self.off, self.b0 = rx_start & 3, rx_start >> 2
        self.rx = rx_start
        self.f = np.full(LW_RING + LW_EXT, -10**9, np.int64)

    def gen(self, n_lo, n_hi):
        """capture_blocks<LW_RING, LW_EXT>(..., b0, (rx + n_lo) >> 2, (rx + n_hi - 1) >> 2)"""
        for b in range((self.rx + n_lo) >> 2, ((self.rx + n_hi - 1) >> 2) + 1):
            pos = red(4 * (b - self.b0))
            samples = 4 * b - self.rx + np.arange(4)
            self.f[pos:pos + 4] = samples
            if pos < LW_EXT:
                self.f[pos + LW_RING:pos + LW_RING + 4] = samples

    def at(self, n):
        return red(n + self.off)


def check_round(ring, rho, L):
    """detection round rho: lane l reads its chunk's positions' window samples [n0, n1 + 47) linearly from ring(n0)"""
    Lc = L - 47
    for lane in range(64):
        n0 = rho * LW_ROUND + lane * LW_CHUNK
        n1 = min(n0 + LW_CHUNK, Lc)
        if n0 >= n1:
            continue
        base = ring.at(n0)
        need = np.arange(n0, n1 + 47)
        assert base + len(need) + 2 <= LW_RING + LW_EXT          # the 80-float block reads stay in the region
        assert np.array_equal(ring.f[base:base + len(need)], need), (rho, lane)


@pytest.mark.parametrize("n_data", [5, 6, 8])
def test_ring_reads_are_the_samples_meant(n_data):
    rng = np.random.default_rng(n_data)
    nfr = 320 + 80 * n_data
    wave_len = 10 * (2 * nfr + 20)
    L = int(0.307 * wave_len)
    R = (L - 47 + LW_ROUND - 1) // LW_ROUND
    assert R == 3
    for _ in range(300):
        rx = int(rng.integers(0, wave_len - L))
        decided = bool(rng.integers(0, 2))
        ring = Ring(rx)
        ring.gen(0, min(L, LW_PIECE))
        check_round(ring, 0, L)
        ring.gen(LW_ROUND, min(L, LW_ROUND + LW_PIECE))
        check_round(ring, 1, L)
        held = 1
        if not decided:
            ring.gen(2 * LW_ROUND, min(L, 2 * LW_ROUND + LW_PIECE))
            check_round(ring, 2, L)
            held = 2
        # a decided front lies below 2 LW_ROUND - 300; a failed sync gives p = 0
        p = 0 if rng.random() < 0.2 else int(rng.integers(11, (2 * LW_ROUND - 300) if decided else L - 60))
        lo, hi = p + 2 * 80 - 20, min(p + 2 * (nfr - 1) + 10, L - 1)   # the first instant read is frame sample 80
        res_hi = min(L, held * LW_ROUND + LW_PIECE)
        res_lo = res_hi + 3 - LW_RING
        if hi >= res_hi:
            ring.gen(max(lo, res_hi), hi + 1)
        elif lo < res_lo:
            ring.gen(lo, min(hi + 1, res_lo))
        # every matched-filter run (instants [80, 112), [192, 320), [336 + 80 d, 400 + 80 d) in runs of MF_RUN) in the
        # capture reads 2 MF_RUN + 19 samples from ring(n_lo), n_lo = p + 2 s0 - 20
        starts = [s for a, e in [(80, 112), (192, 320)] + [(336 + 80 * d, 400 + 80 * d) for d in range(n_data)]
                  for s in range(a, e, MF_RUN)]
        for s0 in starts:
            n_lo = p + 2 * s0 - 20
            if n_lo < 0 or p + 2 * (s0 + MF_RUN - 1) >= L:
                continue                                          # the per-instant path (ring(mc) per sample)
            base = ring.at(n_lo)
            need = np.arange(n_lo, n_lo + 2 * MF_RUN + 19)
            assert np.array_equal(ring.f[base:base + len(need)], need), (p, s0)
        for mc in ((lo, hi, (lo + hi) // 2) if lo <= hi else ()):  # the per-instant path's single reads
            assert ring.f[ring.at(mc)] == mc


def trimmed_passes(bs, be):
    """capture_blocks<RING, EXT, TRIM = true>'s schedule (ofdm_frame.hip): (p0, U) per pass -- whole passes of 4 blocks
    per lane while more than 192 blocks remain, then one pass of ceil(rest / 64) blocks per lane"""
    out, p0 = [], bs
    while be - p0 >= 3 * 64:
        out.append((p0, 4))
        p0 += 4 * 64
    for u, need in ((3, 2 * 64), (2, 64), (1, 0)):
        if be - p0 >= need:
            out.append((p0, u))
            break
    return out


def test_trimmed_passes_store_every_block_once():
    """the matched-filter window's missing end (1..483 blocks): lane l of a pass (p0, U) stores blocks p0 + l + 64 u,
    u < U, that are <= be -- together exactly [bs, be], each once, with ceil(n / 64) blocks per lane in all but whole
    passes (n = be - bs + 1)"""
    for n in range(1, 700):
        bs = 17 + n
        be = bs + n - 1
        stored = []
        lane_blocks = 0
        for p0, u in trimmed_passes(bs, be):
            lane_blocks += u
            stored += [p0 + lane + 64 * k for k in range(u) for lane in range(64) if p0 + lane + 64 * k <= be]
        assert sorted(stored) == list(range(bs, be + 1)), n
        # whole passes for all but the last (n - 1) % 256 + 1 blocks, which take ceil(. / 64) blocks per lane
        assert lane_blocks == 4 * ((n - 1) // 256) + -(-((n - 1) % 256 + 1) // 64), n
        assert lane_blocks <= 4 * -(-n // 256), n                 # never more than whole passes
