// ofdm_symbol.hip -- symbol-mode kernels for gfx950 (MI355X): K1 batched FFT, K2 Tx builder,
// K3 fused AWGN/Rayleigh + receiver chain with counters.  DESIGN.md §2-§4 describe layout,
// roofline and the RNG spec; the per-stage reference lines are cited inline.  The real-noise AWGN
// sweeps (c2/c3/c4, the benchmark) run the packed receivers of ofdm_rxpack.hip instead (launch_rx);
// the kernels here serve complex noise, the 4-tap Rayleigh channel (c5) and noiseless runs.
//
// K1 (the standalone fft()/ifft()) runs one transform per lane quad, staged through LDS (fft64_lds_kernel); the Tx and
// receiver kernels below keep the register mapping:
// ONE LANE OWNS ONE 64-SAMPLE WINDOW (a data symbol or the LTF pair); its 64-point FFT
// lives in that lane's VGPRs (ofdm_device.h).  In LS mode a wave carries 21 frames as lanes
// {E, D0, D1}: the data lanes fetch S = F1 + F2 (OFDM.c:830-850) from their E lane with ds_bpermute.
//
// Register discipline: the first radix-4 stage is fused with sample generation (load + channel +
// noise) four butterflies at a time, then the four 16-point sub-FFTs run one after another and
// each sub-block's bins are consumed (demapped or stored) at once.  sched_fence() pins that order
// and demap_sub pins its EVM chain, so the live set stays ~128 VGPRs + temporaries: 2 waves/SIMD
// without scratch (tools/resource_usage.py).
#include <algorithm>
#include <cstdlib>
#include "ofdm_internal.h"
#include "ofdm_rxcommon.h"

#define OFDM_RX_LS_WAVES 2      // complex-noise / Rayleigh / noiseless LS: 224 VGPRs, no spill (3: 43-55 spilled, same speed)
#define OFDM_RX_IDEAL_WAVES 2   // (3: 25-62 spilled)

namespace ofdm {

// Phase marks of the receivers below (0 window + noise + first radix-4 stage, 1 sub-block FFTs, 2 equaliser
// fetch + demap, 3 frame metrics + counters, 4 group end).  They compile to nothing; the s_memtime build that
// measured them (-DOFDM_RX_STAMPS) is in git history (profiles/r06/README.md).
struct RxStamp {
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(unsigned long long *) {}
};

// ======================================================================== K1: batched FFT
// FOUR LANES (a quad) PER TRANSFORM.  Lane q of the quad holds the 16 samples x[16q + j], then
//   X[4k + r] = sum_j W16^{jk} ( W64^{jr} sum_q x[16q + j] W4^{qr} )     (radix-4 DIF, first stage across lanes)
// the inner 4-point DFT over q runs across the quad as two DPP exchanges (quad_perm xor 2, xor 1), lane q
// ending with output residue r = bitrev2(q); the twiddles W64^{jr} are per-lane constants held in VGPRs;
// the 16-point DFT over j runs in the lane's registers (dif4<16>).  No cross-lane LDS traffic in the
// transform itself, ~29 VALU wave-instructions per transform, so the kernel is HBM-bound.  Earlier K1 forms
// (lane per transform, wavefront per transform with __shfl, the quad kernel with direct HBM access) are in
// git history (profiles/r06/README.md).
template <int CTRL>
__device__ __forceinline__ float2 dpp_f2(float2 v) {
    return make_float2(__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.x), CTRL, 0xF, 0xF, false)),
                       __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.y), CTRL, 0xF, 0xF, false)));
}
// Both HBM sides are coalesced through LDS (round 5): loading each quad lane's 16 B at byte
// 128 q + 16 c of its transform directly would make one wave-instruction touch 64 different 128-B lines (and its
// stores 16 lines in 32-B pieces); round 2's ablation priced perfectly coalesced loads at +9 % for fft
// (profiles/r02/k1q/fft_ab.txt).  Non-temporal stores: +1.7 % (profiles/r05/ab/k1.txt).  A wave
// owns TPW = 8 transforms (4 KB, contiguous in HBM), quads 0..7 (lanes 0..31) transforming them:
//   * loads: TPW / 2 LDS-DMA instructions (global_load_lds_dwordx4), each reading 1 KB of HBM contiguously; the lane ->
//     chunk assignment inside each KB is permuted so that chunk j of transform t lands at slot 32 t + (j ^ s),
//     s = 2 (t & 3) + (j >> 4): then the quad lanes' ds_read_b128 of "chunk 8 q + c" hit 16 distinct 4-bank groups
//     in each of ds_read_b128's 16-lane groups ({0-3, 12-15, 20-27}, ...: transforms t, t + 3, t + 5, t + 6, whose
//     (t & 3) differ) -- no bank conflicts;
//   * the transform (DPP 4-point stage across the quad, per-lane twiddles, 16-point DIF in registers) is the quad
//     kernel's;
//   * stores: bin k of transform t goes to LDS float2 slot 64 t + (k ^ 4 (t & 3)) by ds_write_b64 (the 16 lanes of
//     a 4 x 16 group write 16 distinct bank pairs), then each lane reads back 16 contiguous bytes (ds_read_b128,
//     the XOR keeps a chunk's two bins adjacent) and writes them with one global_store_dwordx4: 1 KB contiguous per
//     wave-instruction.
// 16 KB of LDS per 256-thread block; 87 VGPRs hold it at 5 waves/SIMD.  In place (in == out) is safe: a wave reads all
// its transforms before it writes them.
// Transforms per wave (round 5, profiles/r05/ab/k1.txt): 16 (8 KB per wave, every lane busy) 5.39-5.48e9 transforms/s,
// 8 (4 KB) 5.82-5.84e9 (+7 %), 4 (2 KB, 3/4 of the lanes idle) 4.17e9.  The same shapes as plain copies
// (tools/ubench_copy.hip, profiles/r05/ab/copy_ceiling.txt): 8 KB per wave, loaded whole and then stored, 5.5-5.8 TB/s
// whether staged through LDS or registers and at any occupancy; 4 KB 6.05; 2 KB 6.23; 1 KB 6.27-6.37 TB/s.
#define OFDM_K1_WPE 4       // amdgpu_waves_per_eu lower bound: <= 128 VGPRs (87: 5 waves/SIMD; 6 spill 6 VGPRs)
#define OFDM_K1_TPW 8       // transforms per wave (16: every quad of the wave; 8 / 4: quads 0..TPW-1 only)
static_assert(OFDM_K1_TPW == 16 || OFDM_K1_TPW == 8 || OFDM_K1_TPW == 4, "whole 1-KB load / store instructions");
#define OFDM_K1_LOAD_CPOL 2 // cache-policy bits of the LDS-DMA loads: nt (streamed once; A/B +1.5 % on top of the above)
template <bool INV, int CONV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OFDM_K1_WPE)))
void fft64_lds_kernel(const float2 *in, float2 *out, int64_t n) {   // in == out allowed: not __restrict__
    constexpr int TPW = OFDM_K1_TPW;
    __shared__ __attribute__((aligned(16))) float4 buf[4][32 * TPW];  // per wave: TPW transforms x 32 chunks of 16 B
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t t_base = ((int64_t)blockIdx.x * 4 + wv) * TPW;      // this wave's first transform
    const int64_t avail = (n - t_base) * 32;                           // chunks of this wave that exist (<= 0:
                                                                       // a trailing wave of the last block)
    float4 *wb = buf[wv];
    const float4 *src = reinterpret_cast<const float4 *>(in) + t_base * 32;
#pragma unroll
    for (int i = 0; i < TPW / 2; ++i) {
        const int slot = 64 * i + lane, t = slot >> 5, jp = slot & 31;
        const int j = jp ^ (2 * (t & 3) + (jp >> 4));                  // the chunk whose slot this lane fills
        if (t * 32 + j < avail)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + t * 32 + j),
                                             (__attribute__((address_space(3))) void *)(wb + 64 * i), 16, 0,
                                             OFDM_K1_LOAD_CPOL);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                  // this wave's DMA has landed (wave-private)
    const int q = lane & 3, tl = lane >> 2;                            // quad lane, transform within the wave
    if (TPW == 16 || tl < TPW) {                                       // whole quads idle past TPW
    const int r = ((q & 1) << 1) | (q >> 1);                           // output residue of this lane
    const int64_t t = t_base + tl;
    const float s1 = q < 2 ? 1.0f : -1.0f;
    const float jf = INV ? -1.0f : 1.0f;
    const float2 ca = q == 3 ? make_float2(0.f, jf) : make_float2(q == 1 ? -1.0f : 1.0f, 0.f);
    const float2 cb = q == 2 ? make_float2(0.f, -jf) : make_float2(1.0f, 0.f);
    float2 tw[16];
    static_for<1, 16>([&](auto jc) {
        constexpr int jj = decltype(jc)::value;
        auto w = [](auto ec) {
            constexpr int e = decltype(ec)::value % 64;
            return make_float2(kCos64[e], INV ? kSin64[e] : -kSin64[e]);
        };
        const float2 w1 = w(std::integral_constant<int, jj>{}), w2 = w(std::integral_constant<int, 2 * jj>{}),
                     w3 = w(std::integral_constant<int, 3 * jj>{});
        tw[jj] = r == 1 ? w1 : r == 2 ? w2 : w3;
        if (r == 0) tw[jj] = make_float2(1.0f, 0.0f);
    });
    const float out_scale = INV ? ((r & 1) ? -1.0f / 64.0f : 1.0f / 64.0f) : 1.0f;
    float2 x[64];                                                      // x[j], j < 16 used
    {
        typedef const __attribute__((address_space(3))) f4v lf4c;
        const int sw = 2 * (tl & 3) + (q >> 1);                       // this lane's slot XOR
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const f4v v = *(lf4c *)(wb + 32 * tl + ((8 * q + c) ^ sw));
            x[2 * c] = make_float2(v.x, v.y);
            x[2 * c + 1] = make_float2(v.z, v.w);
        }
    }
    static_for<0, 16>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr float sg = ((!INV || CONV == OFDM_CONV_C) && (j & 1)) ? -1.0f : 1.0f;     // (-1)^n (D5)
        float2 v = make_float2(sg * x[j].x, sg * x[j].y);
        const float2 p2 = dpp_f2<DPP_QUAD_XOR2>(v);
        v = make_float2(fmaf(s1, v.x, p2.x), fmaf(s1, v.y, p2.y));
        const float2 p1 = dpp_f2<DPP_QUAD_XOR1>(v);
        v = make_float2(ca.x * v.x - ca.y * v.y + (cb.x * p1.x - cb.y * p1.y),
                        ca.x * v.y + ca.y * v.x + (cb.x * p1.y + cb.y * p1.x));
        if constexpr (j > 0) v = make_float2(fmaf(v.x, tw[j].x, -v.y * tw[j].y), fmaf(v.x, tw[j].y, v.y * tw[j].x));
        x[j] = v;
    });
    dif4<INV, 16, 0>(x);                                               // bin 4 k' + r at position rev16(k')
    {
        typedef __attribute__((address_space(3))) f2v lf2w;
        lf2w *ob = (lf2w *)wb + 64 * tl;
        const int ox = 4 * (tl & 3);
        static_for<0, 16>([&](auto pc) {
            constexpr int pos = decltype(pc)::value;
            constexpr int kp = ((pos & 3) << 2) | (pos >> 2);          // rev16 is its own inverse
            const float2 v = cscale(x[pos], out_scale);
            f2v w; w.x = v.x; w.y = v.y;
            ob[(4 * kp + r) ^ ox] = w;
        });
    }
    }
    // every lane's bins are in LDS before any lane reads its chunks back (one wave: LDS operations complete in
    // order; the fences keep the compiler from moving the reads above the writes)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float4 *dst = reinterpret_cast<float4 *>(out) + t_base * 32;
#pragma unroll
    for (int i = 0; i < TPW / 2; ++i) {
        const int g = 64 * i + lane, tg = g >> 5, m = g & 31;
        typedef const __attribute__((address_space(3))) f4v lf4c;
        const f4v v = *(lf4c *)(wb + 32 * tg + (m ^ (2 * (tg & 3))));
        if (g < avail) {
            __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(dst) + g);
        }
    }
}

// ======================================================================== K2: Tx builder
// One lane = one data symbol (tx_symbol, ofdm_rxcommon.h: bits -> QPSK -> map + pilots -> ifft -> CP -> HBM).
template <int CONV>
__global__ __launch_bounds__(256, 3) void tx_symbols_kernel(TxArgs a) {
    const int64_t sidx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // symbol within batch
    if (sidx >= a.n_sym) return;
    tx_symbol<CONV>(a, sidx);
}

// ======================================================================== K3: receiver chain
// Where the clean samples of a lane's window come from: sample n (-3..63,
// negative = cyclic prefix, reached only by the 4-tap channel) with a compile-time offset.
// LdsRows: a staged group in LDS (StageGeom), ROW_F2 float2 per row starting at sample R0 - 16;
// base = this lane's column (a data symbol, or the LS receiver's 2T column for the LTF-pair lane).
template <int R0, int ROW_F2>
struct LdsRows {
    lcf2 *base;
    __device__ __forceinline__ void fresh() { opaque(base); }
    template <int N>
    __device__ __forceinline__ float2 at() const { return ld2(base, (N + 16 - R0) * ROW_F2); }
};

// A staged group in LDS: rows R0..79 (R0 = 12 when the 4-tap channel reaches into the CP), each row
// DATA_CHUNKS x 16 B of consecutive symbols followed by EXTRA_CHUNKS x 16 B from a per-row table
// (the LS receiver's 2T column).
template <int CHAN, int DATA_CHUNKS, int EXTRA_CHUNKS>
struct StageGeom {
    static constexpr int R0 = CHAN == OFDM_CHAN_RAYLEIGH4 ? 12 : 16;
    static constexpr int ROWS = SYM_SAMPLES - R0;
    static constexpr int DATA = DATA_CHUNKS;
    static constexpr int ROW_CHUNKS = DATA_CHUNKS + EXTRA_CHUNKS;
    static constexpr int LOADED = ROW_CHUNKS;         // chunks per row filled by LDS-DMA
    static constexpr int ROW_F2 = 2 * ROW_CHUNKS;
    static constexpr int CHUNKS = ROWS * ROW_CHUNKS;
    static constexpr int BUF_F2 = ROWS * ROW_F2;
};

// LS receiver with the 4-tap channel: rows 12..79 of [42 data symbols | 2T chunk | 21 computed
// columns (each frame's 2T (x) h, fade_group) + 1 pad] float2.  One buffer (35.9 KB): 3 blocks/CU.
struct FadeGeom {
    static constexpr int R0 = 12;
    static constexpr int ROWS = SYM_SAMPLES - R0;
    static constexpr int DATA = LS_GROUP_SYMS / 2;
    static constexpr int LOADED = DATA + 1;
    static constexpr int ROW_CHUNKS = LOADED + 11;
    static constexpr int ROW_F2 = 2 * ROW_CHUNKS;
    static constexpr int CHUNKS = ROWS * ROW_CHUNKS;
    static constexpr int BUF_F2 = ROWS * ROW_F2;
    static constexpr int ECOL = 2 * LOADED;            // first computed column
};

// HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: 1 KB per wave-instruction, chunk c lands at LDS
// byte 16 c), spread over the block's 4 waves.  `extra` holds 16 B per table row, row r = window
// sample r - 4 (so staged row `row` uses table row row + R0 - 12).
template <typename G>
__device__ __forceinline__ void stage_group(const RxArgs &a, int64_t col0, float2 *buf, const float2 *extra, int wv,
                                            int lane) {
    const float2 *c0 = a.tx + col0;
    for (int k = wv; k * 64 < G::CHUNKS; k += 4) {
        const int c = k * 64 + lane;
        const int row = c / G::ROW_CHUNKS, j = c - row * G::ROW_CHUNKS;
        if (c < G::CHUNKS && j < G::LOADED) {
            const char *src = j < G::DATA ? (const char *)(c0 + (int64_t)(G::R0 + row) * a.pitch) + j * 16
                                          : (const char *)(extra + 2 * (row + G::R0 - 12));
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)((char *)buf + k * 1024),
                                             16, 0, 0);
        }
    }
}

// The group's demap words (Tx rows 3..6, ofdm_rxcommon.h) into LDS by LDS-DMA: wave wv copies row
// 3 + wv of the n_cols symbols from col0 (4 B per lane, lane l at truth + 4 l).  Columns the DMA does
// not write stay zero (LS E lanes, the idle lane).
__device__ __forceinline__ void stage_truth(const RxArgs &a, int64_t col0, uint32_t *truth /* [4][64] */, int wv,
                                            int lane, int n_cols) {
    if (lane < n_cols) {
        const uint32_t *src = a.bits + (3 + wv) * a.pitch + col0 + lane;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(truth + 64 * wv), 4, 0, 0);
    }
}

// A lane's demap words in LDS, read one sub-block at a time (re-materialised address: the four words
// are not hoisted out of the SNR loop and held across it)
typedef __attribute__((address_space(3))) const uint32_t lcu32;
struct LdsTruth {
    lcu32 *p;    // &truth[0][column]
    template <int R>
    __device__ __forceinline__ uint32_t word() const {
        lcu32 *q = p;
        opaque(q);
        return q[64 * R];
    }
};

// Clean samples n0-3..n0+3 (Rayleigh: the 4-tap channel reaches 3 back) or n0..n0+3 of a lane's window.
template <int CHAN, int N0, typename WS>
__device__ __forceinline__ void rx_load(float2 (&c)[7], const WS &src) {
    // re-materialise per block: keeps LICM from hoisting 16 blocks' worth of addresses
    WS p = src;
    p.fresh();
    if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {
        static_for<0, 7>([&](auto ic) { c[decltype(ic)::value] = p.template at<N0 - 3 + decltype(ic)::value>(); });
    } else {
        static_for<0, 4>([&](auto ic) { c[3 + decltype(ic)::value] = p.template at<N0 + decltype(ic)::value>(); });
    }
}

// Channel + AWGN for samples n0..n0+3 of loaded clean samples c, times (-1)^n (fft() = DFT of
// x(-1)^n, OFDM.c:314-318).  Noise sample at frame time t uses Gaussian t (real) or 2t, 2t+1
// (complex) of the frame's stream; AWGN is real-only as OFDM.c:651 really does (D7).
// K = noise_k(sigma) (real) or noise_k(sigma / sqrt2) (complex): each noisy component is one fma.
// `hd` = philox_head of the frame's noise stream at this SNR point; `tb` = the counter word c2 of
// the window's first Philox block (t0 / 4 real, t0 / 2 complex).
// (The ablation builds that priced each stage, OFDM_ABL_*, are in git history: profiles/r06/README.md.)
// Philox outputs of one group (samples 4g..4g+3 of each quarter): real noise 4 blocks (c2 = tb + g +
// 4i), complex 8 (c2 = tb + 2g + 8i + {0, 1}), computed together with VGPR round keys.
template <int NB>
__device__ __forceinline__ void rx_philox(const PhiloxHead &hd, const uint32_t (&c2)[NB], uint32_t k0, uint32_t k1,
                                          uint4 (&o)[NB]) {
#pragma unroll
    for (int b = 0; b < NB; ++b) o[b] = philox10_c2(hd, c2[b], k0, k1);
}
__device__ __forceinline__ Noise4 rx_noise4(uint4 o, float K) {
    return noise4_of(o, K);
}

// o: the block(s) of samples n0..n0+3 (one for real noise, two for complex)
template <int NOISE, int CHAN, int N0>
__device__ __forceinline__ void rx_noisy(float2 (&x)[64], const float2 (&c)[7], const uint4 *o, float K,
                                         const float2 (&h)[4]) {
    float nr[8], nt[8];     // noise of component j = nr[j] * nt[j]
    if constexpr (NOISE == OFDM_NOISE_REAL) {
        const Noise4 g = rx_noise4(o[0], K);
        nr[0] = g.r0; nt[0] = g.c0; nr[1] = g.r0; nt[1] = g.s0; nr[2] = g.r1; nt[2] = g.c1; nr[3] = g.r1; nt[3] = g.s1;
    } else if constexpr (NOISE == OFDM_NOISE_COMPLEX) {
        const Noise4 g0 = rx_noise4(o[0], K);
        const Noise4 g1 = rx_noise4(o[1], K);
        nr[0] = g0.r0; nt[0] = g0.c0; nr[1] = g0.r0; nt[1] = g0.s0; nr[2] = g0.r1; nt[2] = g0.c1; nr[3] = g0.r1; nt[3] = g0.s1;
        nr[4] = g1.r0; nt[4] = g1.c0; nr[5] = g1.r0; nt[5] = g1.s0; nr[6] = g1.r1; nt[6] = g1.c1; nr[7] = g1.r1; nt[7] = g1.s1;
    }
    static_for<0, 4>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int n = N0 + i;
        float2 y = c[3 + i];
        if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {   // y[t] = sum_l h_l x[t - l], 4 taps < CP
            y = cadd(cadd(cmul(h[0], c[3 + i]), cmul(h[1], c[2 + i])), cadd(cmul(h[2], c[1 + i]), cmul(h[3], c[i])));
        }
        if constexpr (NOISE == OFDM_NOISE_REAL) {
            y.x = fmaf(nr[i], nt[i], y.x);
        } else if constexpr (NOISE == OFDM_NOISE_COMPLEX) {
            y.x = fmaf(nr[2 * i], nt[2 * i], y.x);
            y.y = fmaf(nr[2 * i + 1], nt[2 * i + 1], y.y);
        }
        if constexpr (n & 1) y = make_float2(-y.x, -y.y);
        x[n] = y;
    });
}

// generate the window fused with the first radix-4 stage (4 butterflies per group of 16 samples).
// Pinning the group's LDS reads ahead of its noise generation measured slower (+32 live VGPRs -> more
// spills; the read latency is already hidden by the other 2 waves/SIMD).
template <int NOISE, int CHAN, typename WS>
__device__ __forceinline__ void rx_window_stage1(float2 (&x)[64], const WS &src, uint32_t f_lo,
                                                 uint32_t f_hi, uint32_t t0, uint32_t q, float sigma,
                                                 uint32_t k0, uint32_t k1, const float2 (&h)[4]) {
    const float K = noise_k(NOISE == OFDM_NOISE_COMPLEX ? sigma * INV_SQRT2 : sigma);
    const PhiloxHead hd = philox_head(f_lo, f_hi, STREAM_NOISE | q, k1);     // shared by the 16-32 blocks
    const uint32_t tb = NOISE == OFDM_NOISE_COMPLEX ? t0 >> 1 : t0 >> 2;
    constexpr int NB = NOISE == OFDM_NOISE_COMPLEX ? 8 : NOISE == OFDM_NOISE_REAL ? 4 : 1;
    constexpr int PB = NOISE == OFDM_NOISE_COMPLEX ? 2 : NOISE == OFDM_NOISE_REAL ? 1 : 0;
    // Philox blocks of group g (samples 4g..4g+3 of each quarter)
    auto philox_group = [&](auto gc, uint4 (&o)[NB]) {
        constexpr int g = decltype(gc)::value;
        if constexpr (NOISE != OFDM_NOISE_NONE) {
            // re-materialise per group: keeps LICM from hoisting 16 blocks' worth of round-1 products
            // out of the SNR loop (tb does not depend on the SNR point)
            uint32_t tg = tb;
            opaque(tg);
            uint32_t c2[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b)
                c2[b] = NOISE == OFDM_NOISE_COMPLEX ? tg + 2 * g + 8 * (b >> 1) + (b & 1) : tg + g + 4 * b;
            rx_philox<NB>(hd, c2, k0, k1, o);
        }
    };
    // software pipeline: group g + 1's Philox chains share group g's fence region with its Box-Muller,
    // noise and butterflies (the next group's 16 state VGPRs fit while x is still partly empty).
    // A/B (profiles/r02/ab): c3 -2.0 %, c2 -4.9 % receiver time
    uint4 on[NB];
    philox_group(std::integral_constant<int, 0>{}, on);
    sched_fence();
    static_for<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        float2 c[4][7];
        rx_load<CHAN, 4 * g>(c[0], src);
        rx_load<CHAN, 16 + 4 * g>(c[1], src);
        rx_load<CHAN, 32 + 4 * g>(c[2], src);
        rx_load<CHAN, 48 + 4 * g>(c[3], src);
        uint4 o[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) o[b] = on[b];
        if constexpr (g < 3) philox_group(std::integral_constant<int, g + 1>{}, on);
        rx_noisy<NOISE, CHAN, 4 * g>(x, c[0], o + 0 * PB, K, h);
        rx_noisy<NOISE, CHAN, 16 + 4 * g>(x, c[1], o + 1 * PB, K, h);
        rx_noisy<NOISE, CHAN, 32 + 4 * g>(x, c[2], o + 2 * PB, K, h);
        rx_noisy<NOISE, CHAN, 48 + 4 * g>(x, c[3], o + 3 * PB, K, h);
        static_for<0, 4>([&](auto ic) { dif_stage1<false, 4 * g + decltype(ic)::value>(x); });
        sched_fence();
    });
}

// Shared tail: FFT sub-blocks + demap, per-frame combine of the frame's two data symbols
// (`partner` fetches the other data lane's value), counters.  `leader` lanes (one per valid
// frame) contribute.
template <bool DUMP, int KIND, typename TW, typename HF, typename PF>
__device__ __forceinline__ void finish_symbol(float2 (&x)[64], const TW &truth, HF &&Hof, PF &&partner,
                                              float2 *dump_eq, uint32_t *dump_bits, bool leader,
                                              unsigned long long *slots, RxStamp &sp) {
    SymState st;
    sym_init(st);
    static_for<0, 4>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        dif_sub16<false, R>(x);
        sp.mark(1);
        Hof.template prefetch<R>(x);
        demap_sub<DUMP, R, KIND>(x, truth.template word<R>(), Hof, dump_eq, st);
        sched_fence();
        sp.mark(2);
    });
    if constexpr (DUMP) {
        if (dump_bits) { dump_bits[0] = st.d[0]; dump_bits[1] = st.d[1]; dump_bits[2] = st.d[2]; }
    }
    const float evm = finish_evm<KIND>(st);
    const float e_other = __uint_as_float(partner(__float_as_uint(evm)));
    const uint32_t be_other = partner(st.be), ax_other = partner(st.ax);
    FrameAcc acc;
    frame_metrics(acc, evm + e_other, st.be + be_other, st.ax + ax_other);   // used on leader lanes only
    flush_lanes(acc, leader, slots);
    sp.mark(3);
}

// The 4-tap channel y[n] = sum_l h_l x[n - l] (taps < CP) applied once per staged group instead of
// once per SNR point: it does not depend on the SNR, so the per-SNR loop only adds noise (same fp32
// operations as rx_noisy's per-SNR form).  Wave v computes the outputs n = 16 v .. 16 v + 15 of column
// in_col into column out_col; all inputs are read before any output is written.
template <typename G>
__device__ __forceinline__ void fade_group(float2 *buf, int wv, int in_col, int out_col, bool active,
                                           const float2 (&h)[4]) {
    static_assert(G::R0 == 12, "the channel reaches 3 samples into the cyclic prefix");
    float2 xv[19];       // x[16 v - 3 + k]: window sample n sits in staged row n + 16 - R0
    static_for<0, 19>([&](auto kc) {
        xv[decltype(kc)::value] = buf[(16 * wv + decltype(kc)::value + 1) * G::ROW_F2 + in_col];
    });
    __syncthreads();
    if (active) {
        static_for<0, 16>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const float2 y = cadd(cadd(cmul(h[0], xv[i + 3]), cmul(h[1], xv[i + 2])),
                                  cadd(cmul(h[2], xv[i + 1]), cmul(h[3], xv[i])));
            buf[(16 * wv + i + 4) * G::ROW_F2 + out_col] = y;
        });
    }
    __syncthreads();
}

// ---- LS estimate: a wave carries 21 frames, lanes {E, D0, D1} per frame (lane 63 idle) ----
// H = 0.5 (F1 + F2) conj(Lf) (OFDM.c:830-850) with F1 + F2 = FFT(r1 + r2) (linearity).  Both LTF
// windows hold the same clean samples T, so the E lane transforms 2T (+ channel) plus the pair's
// noise n1 + n2, drawn once as sqrt(2) sigma x the LTF1-slot Gaussians (same law).
// The data lanes fetch S = F1 + F2 from their E lane with ds_bpermute.
//
// The 4 waves of a block share one staged group (42 symbols x 64-68 rows, plus the 2T column)
// in LDS and split the SNR points; the next group is prefetched by LDS-DMA into the other buffer.
template <int CHAN>
using LsGeom = StageGeom<CHAN, LS_GROUP_SYMS / 2, 1>;      // 42 data symbols + the 2T chunk per row
static_assert(LS_ROW_F2 == 2 * (LS_GROUP_SYMS / 2 + 1), "LS staged row = 42 symbols + 2T (x2)");

// S[k] = F1[k] + F2[k] from the frame's E lane (ds_bpermute), fetched for a whole FFT sub-block at
// once; Z = Y / (0.5 Lf S) = 2 Lf Y conj(S) / |S|^2
struct LsBpermuteEq {
    uint32_t e_addr;
    float2 S[16];
    template <int R>
    __device__ __forceinline__ void prefetch(const float2 (&x)[64]) {
        static_for<0, 16>([&](auto kc) {
            constexpr int bin = 4 * decltype(kc)::value + R;
            if constexpr (data_index(bin) >= 0) {
                const float2 Y = x[digit_rev4(bin)];
                S[decltype(kc)::value] = make_float2(
                    __int_as_float(__builtin_amdgcn_ds_bpermute((int)e_addr, __float_as_int(Y.x))),
                    __int_as_float(__builtin_amdgcn_ds_bpermute((int)e_addr, __float_as_int(Y.y))));
            }
        });
    }
    template <typename B>
    __device__ __forceinline__ EqOut<2> operator()(float2 Y, B) const {
        constexpr int bin = B::value;
        const float2 Sb = S[bin >> 2];
        EqOut<2> e;
        e.r = __builtin_amdgcn_rcpf(fmaf(Sb.x, Sb.x, Sb.y * Sb.y));
        e.u = cscale(cmulc(Y, Sb), (float)ltf_sign(bin));
        return e;
    }
};

template <int NOISE, int CHAN, bool DUMP>
__global__ __launch_bounds__(256, OFDM_RX_LS_WAVES) void rx_ls_kernel(RxArgs a) {
    // 4-tap channel: applied once per group (fade_group) into one buffer, then the SNR loop runs the
    // AWGN form; no prefetch of the next group (the LDS holds one fading group per block)
    constexpr bool FADE = CHAN == OFDM_CHAN_RAYLEIGH4;
    constexpr int LCHAN = FADE ? OFDM_CHAN_AWGN : CHAN;
    using G = std::conditional_t<FADE, FadeGeom, LsGeom<CHAN>>;
    constexpr int NBUF = FADE ? 1 : 2;
    __shared__ unsigned long long sacc[OFDM_MAX_SNR][8];
    __shared__ __attribute__((aligned(16))) float2 sbuf[NBUF][G::BUF_F2];
    __shared__ uint32_t struth[NBUF][4][64];
    for (int i = threadIdx.x; i < a.n_snr * 8; i += blockDim.x) (&sacc[0][0])[i] = 0ull;
    for (int i = threadIdx.x; i < NBUF * 4 * 64; i += blockDim.x) (&struth[0][0][0])[i] = 0u;
    __syncthreads();                                   // zero columns before the first truth DMA
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int fr = lane / 3, role = lane - 3 * fr;     // lane 63: fr 21 (no frame), role 0
    const bool is_e = role == 0;
    const int col = is_e ? (FADE ? FadeGeom::ECOL + fr : LS_GROUP_SYMS) : 2 * fr + role - 1;
    // window start on the frame timeline: LTF pair at the LTF1 slots 192, D0 336, D1 416
    const uint32_t t0 = is_e ? 192u : 256u + 80u * (uint32_t)role;
    const uint32_t e_addr = (uint32_t)(3 * fr) << 2;
    const uint32_t d1_addr = (uint32_t)(lane + 1) << 2;
    const int64_t n_groups = (a.n_frames + LS_GROUP_FRAMES - 1) / LS_GROUP_FRAMES;
    [[maybe_unused]] const int64_t P = a.pitch;

    // Groups past the first gridDim.x are handed out from a per-launch atomic counter (a.work), one group
    // ahead of the staging: the block always knows the group it stages next (nxt) and thread 0 fetches
    // the one after it into LDS during the current group; blocks that run fast take more groups.  The LDS
    // slot alternates with the group's parity: a slot is rewritten only after a barrier that follows
    // every read of it.
    __shared__ int next_group[2];
    int par = 0;
    int cur = 0;
    int64_t grp = blockIdx.x;
    if (grp < n_groups) {
        stage_group<G>(a, grp * LS_GROUP_SYMS, sbuf[0], a.ltf2_rows, wv, lane);
        stage_truth(a, grp * LS_GROUP_SYMS, &struth[0][0][0], wv, lane, LS_GROUP_SYMS);
    }
    if (threadIdx.x == 0) next_group[1] = (int)gridDim.x + (int)atomicAdd(a.work, 1ull);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int64_t nxt = __builtin_amdgcn_readfirstlane(next_group[1]);
    RxStamp sp;
    sp.start();
    for (; grp < n_groups;) {
        const int64_t fl = grp * LS_GROUP_FRAMES + fr;
        const bool valid = fr < LS_GROUP_FRAMES && fl < a.n_frames;
        const uint64_t f = a.first_frame + (uint64_t)fl;
        const uint32_t f_lo = (uint32_t)f, f_hi = (uint32_t)(f >> 32);
        float2 h[4] = {make_float2(1.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
        // the group after nxt (read after this group's closing barrier; the previous value was read before it)
        if (threadIdx.x == 0) next_group[par] = (int)gridDim.x + (int)atomicAdd(a.work, 1ull);
        if constexpr (FADE) {
            // lane = staged column: 0..41 the data symbols (in place), 42..62 frame lane - 42's 2T (x) h
            const bool dcol = lane < LS_GROUP_SYMS;
            const int ff = dcol ? lane >> 1 : lane - LS_GROUP_SYMS;
            const uint64_t fg = a.first_frame + (uint64_t)(grp * LS_GROUP_FRAMES + ff);
            float2 hg[4];
            channel_taps((uint32_t)fg, (uint32_t)(fg >> 32), a.k0, a.k1, hg);
            fade_group<G>(sbuf[0], wv, dcol ? lane : LS_GROUP_SYMS, dcol ? lane : FadeGeom::ECOL + ff, lane < 63, hg);
        } else {
            if (nxt < n_groups) {
                stage_group<G>(a, nxt * LS_GROUP_SYMS, sbuf[cur ^ 1], a.ltf2_rows, wv, lane);
                stage_truth(a, nxt * LS_GROUP_SYMS, &struth[cur ^ 1][0][0], wv, lane, LS_GROUP_SYMS);
            }
        }
        LdsRows<G::R0, G::ROW_F2> src;
        src.base = (lcf2 *)(sbuf[FADE ? 0 : cur] + col);
        LdsTruth truth;
        truth.p = (lcu32 *)&struth[FADE ? 0 : cur][0][is_e ? LS_GROUP_SYMS : col];

        for (int q = wv; q < a.n_snr; q += 4) {
            LdsRows<G::R0, G::ROW_F2> s = src;
            uint32_t flo = f_lo, fhi = f_hi;
            float2 hq[4] = {h[0], h[1], h[2], h[3]};
            s.fresh(); opaque(flo); opaque(fhi);
            const float sg = is_e ? a.sigma[q] * 1.41421356237309504880f : a.sigma[q];
            float2 x[64];
            rx_window_stage1<NOISE, LCHAN>(x, s, flo, fhi, t0, (uint32_t)(a.q_base + q), sg, a.k0, a.k1, hq);
            sp.mark(0);
            float2 *dump_eq = nullptr;
            uint32_t *dump_bits = nullptr;
            if constexpr (DUMP) {
                if (!is_e && valid) {
                    const int64_t r = ((int64_t)q * a.dump_frames + fl) * 2 + (role - 1);
                    dump_eq = a.dump_eq + r * 48;
                    dump_bits = a.dump_bits + r * 3;
                }
            }
            LsBpermuteEq Hof;
            Hof.e_addr = e_addr;
            auto partner = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)d1_addr, (int)v); };
            finish_symbol<DUMP, 2>(x, truth, Hof, partner, dump_eq, dump_bits, role == 1 && valid, sacc[q], sp);
        }
        if constexpr (FADE) {
            __syncthreads();                               // every wave is done with the buffer
            if (nxt < n_groups) {
                stage_group<G>(a, nxt * LS_GROUP_SYMS, sbuf[0], a.ltf2_rows, wv, lane);
                stage_truth(a, nxt * LS_GROUP_SYMS, &struth[0][0][0], wv, lane, LS_GROUP_SYMS);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next group landed
        __syncthreads();                                   // and every wave is done with this one
        sp.mark(4);
        cur ^= 1;
        grp = nxt;
        nxt = __builtin_amdgcn_readfirstlane(next_group[par]);
        par ^= 1;
    }
    sp.flush(a.stamps);
    block_flush(a, sacc);
}

// ---- ideal channel knowledge: every lane a data symbol ----
// A block stages 64 consecutive symbols (rows R0..79, 32-34 KB, one buffer: three blocks per CU hide
// each other's staging) and its 4 waves split the SNR points over them.
template <int CONV, int NOISE, int CHAN, bool DUMP>
__global__ __launch_bounds__(256, OFDM_RX_IDEAL_WAVES) void rx_ideal_kernel(RxArgs a) {
    constexpr bool FADE = CHAN == OFDM_CHAN_RAYLEIGH4;     // channel applied once per group (fade_group)
    constexpr int LCHAN = FADE ? OFDM_CHAN_AWGN : CHAN;
    using G = StageGeom<CHAN, 32, 0>;
    __shared__ unsigned long long sacc[OFDM_MAX_SNR][8];
    __shared__ __attribute__((aligned(16))) float2 sbuf[G::BUF_F2];
    __shared__ uint32_t struth[4][64];
    for (int i = threadIdx.x; i < a.n_snr * 8; i += blockDim.x) (&sacc[0][0])[i] = 0ull;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int d = lane & 1;
    const uint32_t t0 = 336u + 80u * (uint32_t)d;
    const int64_t n_groups = (2 * a.n_frames + 63) / 64;
    [[maybe_unused]] const int64_t P = a.pitch;
    RxStamp sp;
    sp.start();
    for (int64_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {
        stage_group<G>(a, grp * 64, sbuf, nullptr, wv, lane);
        stage_truth(a, grp * 64, &struth[0][0], wv, lane, 64);
        const uint32_t so = (uint32_t)(grp * 64 + lane);
        const int64_t fl = (int64_t)(so >> 1);
        const bool valid = fl < a.n_frames;
        const uint64_t f = a.first_frame + (uint64_t)fl;
        const uint32_t f_lo = (uint32_t)f, f_hi = (uint32_t)(f >> 32);
        float2 h[4] = {make_float2(1.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
        if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) channel_taps(f_lo, f_hi, a.k0, a.k1, h);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                                   // the group has landed for every wave
        if constexpr (FADE) fade_group<G>(sbuf, wv, lane, lane, true, h);   // column = lane, its frame's taps
        LdsRows<G::R0, G::ROW_F2> src;
        src.base = (lcf2 *)(sbuf + lane);
        LdsTruth truth;
        truth.p = (lcu32 *)&struth[0][lane];
        for (int q = wv; q < a.n_snr; q += 4) {
            LdsRows<G::R0, G::ROW_F2> s = src;
            uint32_t flo = f_lo, fhi = f_hi;
            float2 hq[4] = {h[0], h[1], h[2], h[3]};
            s.fresh(); opaque(flo); opaque(fhi);
            if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {
                static_for<0, 4>([&](auto lc) { opaque(hq[decltype(lc)::value].x); opaque(hq[decltype(lc)::value].y); });
            }
            float2 x[64];
            rx_window_stage1<NOISE, LCHAN>(x, s, flo, fhi, t0, (uint32_t)(a.q_base + q), a.sigma[q], a.k0, a.k1, hq);
            sp.mark(0);
            float2 *dump_eq = nullptr;
            uint32_t *dump_bits = nullptr;
            if constexpr (DUMP) {
                if (valid) {
                    const int64_t r = ((int64_t)q * a.dump_frames + fl) * 2 + d;
                    dump_eq = a.dump_eq + r * 48;
                    dump_bits = a.dump_bits + r * 3;
                }
            }
            constexpr int KIND = CHAN == OFDM_CHAN_AWGN ? 0 : 1;
            auto Hof = [&](float2 Y, auto binc) {
                constexpr int bin = decltype(binc)::value;
                constexpr float cs = (CONV == OFDM_CONV_C && (bin & 1)) ? -1.0f : 1.0f;
                EqOut<KIND> e;
                if constexpr (CHAN == OFDM_CHAN_AWGN) {
                    e.u = cscale(Y, cs);
                } else {
                    float2 H = hq[0];
                    H = csub(H, twiddle<bin * 1, false>(hq[1]));     // e^{-j2pi(i-32)l/64} = (-1)^l W^{il}
                    H = cadd(H, twiddle<bin * 2, false>(hq[2]));
                    H = csub(H, twiddle<bin * 3, false>(hq[3]));
                    e.r = __builtin_amdgcn_rcpf(fmaf(H.x, H.x, H.y * H.y));
                    e.u = cscale(cmulc(Y, H), cs);                  // Y / (cs H) = cs Y conj(H) / |H|^2
                }
                return e;
            };
            auto partner = [](uint32_t v) { return dpp_u<DPP_QUAD_XOR1>(v); };
            auto eq = eq_fn(Hof);
            finish_symbol<DUMP, KIND>(x, truth, eq, partner, dump_eq, dump_bits, d == 0 && valid, sacc[q], sp);
        }
        __syncthreads();                                   // every wave is done with the group
        sp.mark(4);
    }
    sp.flush(a.stamps);
    block_flush(a, sacc);
}

// ======================================================================== launchers
// (16 lanes per transform at 2 KB per wave, fft64_row_kernel: correct and LDS-conflict-free but -10 %, round 6,
// profiles/r06/k1/ab_rows.txt; in history at commit f61d0a7)
template <bool INV>
static void launch_fft_conv(int conv, hipStream_t st, const float2 *in, float2 *out, int64_t n) {
    const dim3 gl((unsigned)((n + 4 * OFDM_K1_TPW - 1) / (4 * OFDM_K1_TPW)));
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL((fft64_lds_kernel<INV, OFDM_CONV_C>), gl, dim3(256), 0, st, in, out, n);
    else hipLaunchKernelGGL((fft64_lds_kernel<INV, OFDM_CONV_MATLAB>), gl, dim3(256), 0, st, in, out, n);
}

void launch_fft64(hipStream_t st, const float2 *in, float2 *out, int64_t n, int inverse, int conv) {
    if (inverse) launch_fft_conv<true>(conv, st, in, out, n);
    else launch_fft_conv<false>(OFDM_CONV_C, st, in, out, n);
}

void launch_tx(hipStream_t st, const TxArgs &a, int conv) {
    const dim3 g((unsigned)((a.n_sym + 255) / 256));
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL(tx_symbols_kernel<OFDM_CONV_C>, g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(tx_symbols_kernel<OFDM_CONV_MATLAB>, g, dim3(256), 0, st, a);
}

template <int NOISE, int CHAN, bool DUMP>
static void launch_rx_t(hipStream_t st, const RxArgs &a, int est, int conv, unsigned grid) {
    if (est == OFDM_EST_LS) {
        hipLaunchKernelGGL((rx_ls_kernel<NOISE, CHAN, DUMP>), dim3(grid), dim3(256), 0, st, a);
    } else if (conv == OFDM_CONV_C) {
        hipLaunchKernelGGL((rx_ideal_kernel<OFDM_CONV_C, NOISE, CHAN, DUMP>), dim3(grid), dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL((rx_ideal_kernel<OFDM_CONV_MATLAB, NOISE, CHAN, DUMP>), dim3(grid), dim3(256), 0, st, a);
    }
}

template <int NOISE, bool DUMP>
static void launch_rx_n(hipStream_t st, const RxArgs &a, int est, int conv, int chan, unsigned grid) {
    if (chan == OFDM_CHAN_AWGN) launch_rx_t<NOISE, OFDM_CHAN_AWGN, DUMP>(st, a, est, conv, grid);
    else launch_rx_t<NOISE, OFDM_CHAN_RAYLEIGH4, DUMP>(st, a, est, conv, grid);
}

void launch_rx(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid) {
    if (rx_pack_applies(cfg)) {
        launch_rx_pack(st, a, cfg, dump, grid);
        return;
    }
    if (dump) {
        switch (cfg.noise) {
            case OFDM_NOISE_REAL: launch_rx_n<OFDM_NOISE_REAL, true>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
            case OFDM_NOISE_COMPLEX: launch_rx_n<OFDM_NOISE_COMPLEX, true>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
            default: launch_rx_n<OFDM_NOISE_NONE, true>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
        }
    } else {
        switch (cfg.noise) {
            case OFDM_NOISE_REAL: launch_rx_n<OFDM_NOISE_REAL, false>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
            case OFDM_NOISE_COMPLEX: launch_rx_n<OFDM_NOISE_COMPLEX, false>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
            default: launch_rx_n<OFDM_NOISE_NONE, false>(st, a, cfg.est, cfg.conv, cfg.channel, grid); break;
        }
    }
}

int rx_grid(const ofdm_cfg &cfg, int64_t n_frames, int device) {
    if (rx_pack_applies(cfg)) return rx_pack_grid(cfg, n_frames, device);
    // LS: one block per 21-frame group in flight; ideal: one wave per 64 symbols, 4 waves per block
    // one block per staged group in flight (LS: 21 frames, ideal: 64 symbols)
    const int64_t need = cfg.est == OFDM_EST_LS ? (n_frames + LS_GROUP_FRAMES - 1) / LS_GROUP_FRAMES
                                                : (2 * n_frames + 63) / 64;
    int per_cu = 0, cus = 0;
    const void *k = cfg.est == OFDM_EST_LS
        ? (cfg.channel == OFDM_CHAN_AWGN
               ? reinterpret_cast<const void *>(&rx_ls_kernel<OFDM_NOISE_REAL, OFDM_CHAN_AWGN, false>)
               : reinterpret_cast<const void *>(&rx_ls_kernel<OFDM_NOISE_REAL, OFDM_CHAN_RAYLEIGH4, false>))
        : reinterpret_cast<const void *>(&rx_ideal_kernel<OFDM_CONV_C, OFDM_NOISE_REAL, OFDM_CHAN_AWGN, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
    const int64_t cap = (int64_t)per_cu * cus;
    const int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace ofdm
