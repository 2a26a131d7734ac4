// ofdm_frame.hip -- frame mode: the reference's own trial on gfx950.
//
//   K4a frame_wave_kernel : Transmitter() (OFDM.c:467-618) -- preambles + data symbols, 2x zero
//                           stuffing, 21-tap RRC, x10 repeat, mean power (OFDM.c:637-643).
//   K4b frame_sync_kernel : one 128-thread block per (trial, SNR) item: capture (OFDM.c:945-955) + real
//                           AWGN (OFDM.c:651) in LDS, Packet_Detection (659-683) as fma-chained sliding
//                           sums with sign-bit crossings, Packet_Selection (685-771) as a DPP prefix max
//                           + block min/max, the RRC matched filter only at the down-sampled instants the
//                           receiver reads (965, 984-996), coarse/fine CFO (773-828) on wave 0, and the
//                           rotated LTF / data windows handed to
//   K4b' frame_sym_kernel : the same register FFT + LS estimate + demap as symbol mode (830-1165).
//   K4c ota_kernel        : Transmission_Over_Air() on a caller-provided waveform.
//
// The capture lives in LDS (24 KB per trial for the reference's 2-symbol message; frames carry 1..8
// data symbols, ofdm_set_message); detection keeps only the >0.75 crossings as a bit mask, since
// Packet_Selection needs nothing else (it re-reads Corr_Out only at front+230).
#include "ofdm_internal.h"
#include "ofdm_ctx.h"
#include "ofdm_rxcommon.h"
#include <cmath>
#include <cstring>
#include <vector>

namespace ofdm {

// frame geometry for nd data symbols (OFDM.c:569-612, 945): [STF 160 | LTF 160 | nd x 80]
constexpr int FR_MAX_DATA = MSG_MAX_FRAMES;
constexpr int FR_MAX = 320 + 80 * FR_MAX_DATA;
constexpr int FR_REPS = 10;                  // OFDM.c:607-612
constexpr double TS = 1.0 / 20e6;            // OFDM.c:16-17
__host__ __device__ constexpr int fr_len(int nd) { return 320 + 80 * nd; }
__host__ __device__ constexpr int wave_len_for(int nd) { return (2 * fr_len(nd) + 20) * FR_REPS; }   // 2x + RRC tail
inline int cap_len_for(int nd) { return (int)(wave_len_for(nd) * 0.307); }                          // OFDM.c:945
constexpr int CAP_ABS_MAX = 6000;            // LDS budget of the capture (>= cap_len_for(FR_MAX_DATA) = 5955)

// short training tones S_k at bins 6..58 (OFDM.c:483-490): +-1 on every 4th tone, times (1+j)
__host__ __device__ constexpr int stf_sign(int bin) {
    constexpr int8_t S[53] = {0, 0, 1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 0,
                              0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0};
    return (bin >= 6 && bin <= 58) ? S[bin - 6] : 0;
}

struct WaveArgs {
    float2 *wave;        // [wave_len_for(n_data)]
    double *power;       // mean |x|^2 over the waveform
    uint32_t table[3 * FR_MAX_DATA];   // payload words of the data symbols
    int32_t n_data;
    float taps[21];
    float stf_scale;     // sqrt(13/6) as the float of OFDM.c:479
};

struct FrameArgs {
    const float2 *wave;        // repeated frame waveform (K4a or caller data)
    const float2 *ext;         // external capture (ofdm_receiver), used for item 0 when non-null
    uint64_t first_trial;
    int64_t n_trials;
    int32_t n_snr, q_base;
    int32_t cap_len, float_cfo, matlab, fixed_start, noise, wave_len, n_data, word_stats;
    int32_t fr_in_cap;              // fr[] inside the capture region (fr_in_capture)
    uint32_t k0, k1;
    uint32_t table[3 * FR_MAX_DATA];
    uint32_t dtable[4 * FR_MAX_DATA];   // demap words of the payload symbols (ofdm_rxcommon.h)
    unsigned long long *counters;   // [n_snr][OFDM_NCOUNTERS]
    int32_t *pidx_out;              // [n_snr][n_trials] or null
    // per-trial debug outputs of item 0 (ofdm_receiver), all optional
    float *dbg_res;                 // EVM_dB pre, EVM_dB post, BER
    int32_t *dbg_ints;              // packet_idx, sync_fail, oob, rx_start
    uint32_t *dbg_bits;             // 3 words (96 bits, MSB first) per data symbol
    float2 *dbg_eq;                 // 48 equalised subcarriers per data symbol
    float *dbg_corr;                // Corr_Out (cap_len - 47)
    float2 *dbg_frame;              // fr_len(n_data) samples after fine CFO
    float taps[21];
    float sigma[OFDM_MAX_SNR];
    unsigned long long *stamps;     // OFDM_FRAME_STAMPS builds: cycles per receiver phase [8]
    // sync -> symbol hand-off (one chunk of items; item g = trial (g / n_snr), SNR (g % n_snr))
    int64_t item0, n_items;         // first global item of the chunk, items in it
    float2 *win;                    // hand-off tiles (win_at): LTF1, LTF2, data windows after CFO
    int32_t ipb;                    // items per frame_sym_kernel block = items per hand-off tile
    int4 *info;                     // [n_items]: packet_idx, sync_fail, oob, rx_start
    int32_t add_totals;             // 1 on the last chunk: add frames / symbols / bits / terms
    unsigned long long *work;       // sync kernel: items handed out past the first gridDim.x (zeroed per launch)
};

#ifdef OFDM_FRAME_STAMPS   // diagnostic build: s_memtime per phase, summed over the grid
#define FR_STAMP(k)                                                                  \
    do {                                                                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
        if (threadIdx.x == 0) stamp_acc[k] += t_ - stamp_t;                          \
        stamp_t = t_;                                                                \
    } while (0)
#else
#define FR_STAMP(k) do { } while (0)
#endif

// ======================================================================== K4a: waveform
template <int CONV>
__global__ __launch_bounds__(256) void frame_wave_kernel(WaveArgs a) {
    __shared__ float2 T[2 + FR_MAX_DATA][64];   // STF, LTF, data time symbols
    __shared__ float2 fr[FR_MAX];
    __shared__ double red[256];
    const int tid = threadIdx.x;
    const int nfr = fr_len(a.n_data), nos = 2 * nfr, nfilt = nos + 20;
    if (tid < 2 + a.n_data) {
        const int ds = tid < 2 ? 0 : tid - 2;
        const uint32_t w[3] = {a.table[3 * ds], a.table[3 * ds + 1], a.table[3 * ds + 2]};
        float2 X[64];
        static_for<0, 64>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr float sgn = (CONV == OFDM_CONV_C && (i & 1)) ? -1.0f : 1.0f;   // D5
            const float2 data = tx_bin<CONV, i>(w);
            const float s = sgn * a.stf_scale * (float)stf_sign(i);
            const float2 v = tid == 0 ? make_float2(s, s)                                   // (1+j) S_k scale
                           : tid == 1 ? make_float2(sgn * (float)ltf_sign(i), 0.f)          // L_k
                           : data;
            X[i] = v;
        });
        fft64<true>(X);
        static_for<0, 64>([&](auto nc) {
            constexpr int n = decltype(nc)::value;
            T[tid][n] = cscale(X[digit_rev4(n)], (n & 1) ? -1.0f / 64.0f : 1.0f / 64.0f);
        });
    }
    __syncthreads();
    // frame = [S(160) L(160) D_0(80) .. D_{nd-1}(80)] (OFDM.c:569-583); short = first 16 samples x10,
    // long = [T(32:64) T T] (Preamble_Generator, OFDM.c:392-398), data = [x(48:64) x] (559-565)
    for (int n = tid; n < nfr; n += blockDim.x) {
        float2 v;
        if (n < 160) v = T[0][n & 15];
        else if (n < 320) v = T[1][(n - 160 + 32) & 63];
        else {
            const int d = (n - 320) / 80, j = (n - 320) % 80;
            v = T[2 + d][j < 16 ? 48 + j : j - 16];
        }
        fr[n] = v;
    }
    __syncthreads();
    double pw = 0.0;
    for (int k = tid; k < nfilt; k += blockDim.x) {
        // Convolution(oversampled frame, RRC) (OFDM.c:342-364); odd taps of the zero-stuffed input vanish
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 21; ++j) {
            const int m = k - j;
            if (m >= 0 && m < nos && !(m & 1)) {
                const float2 x = fr[m >> 1];
                acc.x = fmaf(a.taps[j], x.x, acc.x);
                acc.y = fmaf(a.taps[j], x.y, acc.y);
            }
        }
        for (int r = 0; r < FR_REPS; ++r) a.wave[k + r * nfilt] = acc;
        pw += (double)acc.x * acc.x + (double)acc.y * acc.y;
    }
    red[tid] = pw;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    if (tid == 0) *a.power = red[0] / nfilt;      // mean over 10 identical repeats
}

// ======================================================================== K4c: over the air
// Transmission_Over_Air (OFDM.c:635-655): P = mean|x|^2, sigma^2 = P/10^(snr/10), real-only noise
// (D7), Gaussian k of stream (seed, trial, snr_index).
__global__ __launch_bounds__(256) void power_kernel(const float2 *x, int n, double *out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double)x[i].x * x[i].x + (double)x[i].y * x[i].y;
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = blockDim.x / 2; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0] / n;
}

__global__ __launch_bounds__(256) void ota_kernel(const float2 *x, float2 *y, int n, const double *power,
                                                  double snr_lin, uint32_t t_lo, uint32_t t_hi, uint32_t q,
                                                  uint32_t k0, uint32_t k1) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;     // one Philox block = 4 samples
    if (4 * b >= n) return;
    const float sigma = (float)sqrt(*power / snr_lin);
    // the same fp32 arithmetic as frame_sync_kernel's capture, so one stream gives one capture
    const Noise4 nz = noise4_of(philox10(t_lo, t_hi, (uint32_t)b, STREAM_NOISE | q, k0, k1), noise_k(sigma));
    const float zr[4] = {nz.r0, nz.r0, nz.r1, nz.r1}, zc[4] = {nz.c0, nz.s0, nz.c1, nz.s1};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = 4 * b + j;
        if (k < n) {
            float2 v = x[k];
            v.x = fmaf(zr[j], zc[j], v.x);
            y[k] = v;
        }
    }
}

// ======================================================================== K4b: receiver
__device__ __forceinline__ float wave_sum_f(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
}
// wave-uniform max / min of an int: DPP within each row of 16 lanes (quad xor 1, xor 2, half-row and
// row mirrors), then the four row results by readlane -- no LDS round trips (a __shfl_xor ladder is six
// serial ds_bpermute)
template <bool MAX>
__device__ __forceinline__ int wave_ext_i(int v) {
    auto f = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    v = f(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
    v = f(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
    v = f(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));
    v = f(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false));
    return f(f(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             f(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wave_max_i(int v) { return wave_ext_i<true>(v); }
__device__ __forceinline__ int wave_min_i(int v) { return wave_ext_i<false>(v); }
// inclusive prefix max over the wave's lanes (v >= -1): row_shr 1, 2, 4, 8 within each row, then
// row_bcast 15 / 31 carry row results into the later rows; lanes without a source keep -1
__device__ __forceinline__ int wave_prefix_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xC, 0xF, false));
    return v;
}
// the previous lane's value (-1 for lane 0): DPP wave_shr:1
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xF, 0xF, false); }

__device__ __forceinline__ float wave_min_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Word_Optimization_Analysis of one capture (OFDM.c:38-73): RRC matched filter over all n + 20
// outputs (Convolution, OFDM.c:342-364), min / max of the real and imaginary parts -> out[0..1]
__global__ __launch_bounds__(256) void word_length_kernel(const float2 *x, int n, FrameArgs a, float *out) {
    __shared__ float smin[4], smax[4];
    float mn = 1e9f, mx = -1e9f;
    for (int k = threadIdx.x; k < n + 20; k += blockDim.x) {
        float2 v = make_float2(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 21; ++j) {
            const int m = k - j;
            if (m >= 0 && m < n) {
                v.x = fmaf(x[m].x, a.taps[j], v.x);
                v.y = fmaf(x[m].y, a.taps[j], v.y);
            }
        }
        mn = fminf(mn, fminf(v.x, v.y));
        mx = fmaxf(mx, fmaxf(v.x, v.y));
    }
    mn = wave_min_f(mn);
    mx = wave_max_f(mx);
    if ((threadIdx.x & 63) == 0) { smin[threadIdx.x >> 6] = mn; smax[threadIdx.x >> 6] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = fminf(fminf(smin[0], smin[1]), fminf(smin[2], smin[3]));
        out[1] = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    }
}

__device__ __forceinline__ bool bit_at(const unsigned long long *m, int i) { return (m[i >> 6] >> (i & 63)) & 1ull; }
// any set bit in [lo, hi] (inclusive, lo >= 0)
__device__ __forceinline__ bool any_bits(const unsigned long long *m, int lo, int hi) {
    for (int wd = lo >> 6; wd <= (hi >> 6); ++wd) {
        unsigned long long w = m[wd];
        if (wd == (lo >> 6)) w &= ~0ull << (lo & 63);
        if (wd == (hi >> 6) && (hi & 63) != 63) w &= (1ull << ((hi & 63) + 1)) - 1ull;
        if (w) return true;
    }
    return false;
}

// rotate by exp(-j 2 pi f Ts i): phase in revolutions evaluated in fp64 and range-reduced, so the
// rotation matches OFDM.c:802,825 (double cexp of a float frequency) to fp32 rounding
__device__ __forceinline__ float2 cfo_rot(float2 v, double f_ts, int i) {
    const double rev = -f_ts * (double)i;
    const float fr = (float)(rev - rint(rev));
    float s, c;
    // v_sin/v_cos take revolutions; |fr| <= 0.5 is inside their accurate range, and one
    // transcendental each replaces sincospif's range reduction and polynomials (+6 % frame mode)
    s = __builtin_amdgcn_sinf(fr);
    c = __builtin_amdgcn_cosf(fr);
    return make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
}

// Hand-off layout: tiles of ipb items (one frame_sym_kernel block), each tile [64 samples][ipb items][nw
// windows] float2, so that a symbol-kernel wave reading sample n of its lanes' windows reads one
// contiguous row segment (its 16 items x 4 windows = 512 B for the reference frame), where an item-major
// layout made every lane's 8-byte load a different cache line.
__host__ __device__ inline float2 *win_item(float2 *win, int ipb, int nw, int64_t item) {
    const int64_t tile = item / ipb, it = item - tile * ipb;
    return win + tile * 64 * (int64_t)(ipb * nw) + it * nw;      // sample n of window w at [n * ipb * nw + w]
}

// j-th frame sample the receiver reads (j < 160 + 64 nd): the coarse-CFO lag window [80, 112)
// (OFDM.c:786-792), LTF1 + LTF2 [192, 320) (809-815, 830-850), data symbol d's FFT window [336 + 80 d, +64)
__device__ __forceinline__ int needed_k(int j) {
    if (j < 32) return 80 + j;
    if (j < 160) return 160 + j;
    const int e = j - 160;
    return 336 + 80 * (e >> 6) + (e & 63);
}

// ---------------------------------------------------------------- K4b: sync (one block per item)
// LDS image of one trial (dynamic shared memory, sized per launch by frame_lds_bytes)
#ifndef FRAME_SYNC_THREADS
#define FRAME_SYNC_THREADS 128
#endif
constexpr int SYNC_THREADS = FRAME_SYNC_THREADS;   // the waves that share each trial's latency-bound phases
constexpr int SYNC_WAVES = SYNC_THREADS / 64;
static_assert(SYNC_WAVES >= 2 && SYNC_WAVES <= 4, "block reductions use 2..4 waves");
// per-item scratch words after the accumulators: floats [0, 8) (block float sums), ints [8, 32)
constexpr int RED_WORDS = 32, RED_I_MAX = 0, RED_I_PREFIX = 4, RED_I_MINMAX = 8, RED_I_NEXT = 20;
#ifndef FRAME_ITEM_RUN
#define FRAME_ITEM_RUN 4            // items per hand-out of the sync kernel's work counter
#endif
constexpr int ACC_SLOTS = 12;       // per-SNR block accumulators: 9 counter sums + word-length min / max
__host__ __device__ inline int cross_words(int cap_len) { return (cap_len - 47 + 63) / 64 + 1; }
// capture region: cap_len + 8 samples, the capture starting at sample (rx_start & 3) so that every
// Philox block of 4 samples is a 16-byte aligned pair of ds_write_b128
__host__ __device__ inline int cap_region(int cap_len) { return (cap_len + 8 + 1) & ~1; }
// The filtered frame fr[] goes into the part of the capture region the matched filter does not read:
// it reads 2 nfr + 19 samples, so the unread prefix or suffix holds nfr samples whenever the region has
// 4 nfr + 19 (every default capture).  Shorter user captures get fr[] after the scratch words instead.
// (-3.8 KB per trial for the reference capture: 6 instead of 5 blocks per CU.)
__host__ __device__ inline bool fr_in_capture(int cap_len, int n_data) {
    return cap_region(cap_len) >= 4 * fr_len(n_data) + 20;
}
__host__ __device__ inline size_t frame_lds_bytes(int cap_len, int n_data, int n_snr) {
#ifdef OFDM_FR_SEPARATE
    const bool in_cap = false;
#else
    const bool in_cap = fr_in_capture(cap_len, n_data);
#endif
    return (size_t)cap_region(cap_len) * 8 + (size_t)cross_words(cap_len) * 8 + (size_t)n_snr * ACC_SLOTS * 8 +
           RED_WORDS * 4 + (in_cap ? 0 : (size_t)fr_len(n_data) * 8);
}

// block-wide exchange over the SYNC_WAVES waves, the wave partials combined in wave order
// (min of a, max of b) over the waves in one exchange (scratch: 2 SYNC_WAVES slots).  LEAD: the barrier
// that keeps the slots from being overwritten while an earlier exchange still reads them; the item
// loop's slots were last read before the previous item's closing barrier, so it passes false.
template <bool LEAD = true>
__device__ __forceinline__ int2 block_minmax_i(int a, int b, int *red) {
    a = wave_min_i(a);
    b = wave_max_i(b);
    if (LEAD) __syncthreads();
    if ((threadIdx.x & 63) == 0) { red[2 * (threadIdx.x >> 6)] = a; red[2 * (threadIdx.x >> 6) + 1] = b; }
    __syncthreads();
    int2 t = make_int2(red[0], red[1]);
#pragma unroll
    for (int w = 1; w < SYNC_WAVES; ++w) { t.x = min(t.x, red[2 * w]); t.y = max(t.y, red[2 * w + 1]); }
    return t;
}

#ifndef FRAME_SYNC_MINB
#define FRAME_SYNC_MINB 3   // 3 waves/SIMD: +1.3 % (profiles/r01/ab/ab_frame_sync3.json)
#endif
__global__ __launch_bounds__(SYNC_THREADS, FRAME_SYNC_MINB) void frame_sync_kernel(FrameArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int L = a.cap_len, Lc = L - 47;       // Packet_Detection length (OFDM.c:663)
    const int nfr = fr_len(a.n_data);
    const int tid = threadIdx.x, lane = tid & 63;
    float2 *rbase = reinterpret_cast<float2 *>(smem);
    unsigned long long *cross = reinterpret_cast<unsigned long long *>(rbase + cap_region(L));
    unsigned long long *acc = cross + cross_words(L);
    float *redf = reinterpret_cast<float *>(acc + a.n_snr * ACC_SLOTS);
    int *redi = reinterpret_cast<int *>(redf + 8);
    float2 *const fr_sep = reinterpret_cast<float2 *>(redf + RED_WORDS);   // used when !fr_in_capture
    float2 *fr = fr_sep;
    for (int i = tid; i < a.n_snr * ACC_SLOTS; i += SYNC_THREADS) {
        const int k = i % ACC_SLOTS;
        acc[i] = k == 10 ? (unsigned long long)INT64_MAX : k == 11 ? (unsigned long long)INT64_MIN : 0ull;
    }
    // detection positions per lane (< 300, <= 64); odd, so the lanes' 8-byte LDS reads fall in
    // distinct banks
    const int chunk = ((Lc + SYNC_THREADS - 1) / SYNC_THREADS) | 1;
#ifdef OFDM_FRAME_STAMPS
    unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long stamp_t = __builtin_amdgcn_s_memtime();
#endif
    // Items go out in runs of FRAME_ITEM_RUN: block b starts with run b, the runs past the first gridDim.x
    // come from a per-launch atomic counter, so blocks that run fast take more runs.  Thread 0 fetches the
    // next run at the first item of the current one (its wait on the atomic is paid once per run), every
    // thread reads it after the capture barrier of the run's last item.  One atomic per item serialises on
    // the counter's address at ~10 M/s, below the kernel's item rate.
#ifndef OFDM_FRAME_STATIC_ITEMS
    int64_t run_end = (int64_t)blockIdx.x * FRAME_ITEM_RUN + FRAME_ITEM_RUN;
    for (int64_t i = run_end - FRAME_ITEM_RUN, inext = 0; i < a.n_items; i = inext) {
#else
    for (int64_t i = blockIdx.x, inext = 0; i < a.n_items; i = inext) {
#endif
#ifndef FRAME_HOIST_LANE
        // lane-derived values (addresses, sample indices, fp64 instants) are re-derived per item instead of
        // being hoisted out of the item loop and held in ~40 VGPRs across every phase
        int tid = threadIdx.x;
        opaque(tid);
        const int lane = tid & 63;
#endif
#ifndef FRAME_HOIST_ARGS
        // the kernel arguments are re-read per item (scalar loads from the kernarg segment through a pointer
        // made opaque here) instead of being hoisted into ~100 SGPRs held across the item loop, most of
        // which spilled to VGPR lanes and came back by v_readlane (a VALU op) at every use
        using KArgs = const __attribute__((address_space(4))) FrameArgs;
        KArgs *ap = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        KArgs &a = *ap;
#endif
#ifndef OFDM_FRAME_STATIC_ITEMS
        if (threadIdx.x == 0 && i == run_end - FRAME_ITEM_RUN)
            redi[RED_I_NEXT] = (int)gridDim.x + (int)atomicAdd(a.work, 1ull);
#endif
        const int64_t g = a.item0 + i;
        int q;
        int64_t ti;
        if ((uint64_t)g >> 32 == 0) {        // 32-bit division while it fits (~120 SALU less per item)
            const uint32_t g32 = (uint32_t)g, d = (uint32_t)a.n_snr;
            ti = g32 / d;
            q = (int)(g32 - (uint32_t)ti * d);
        } else {
            q = (int)(g % a.n_snr);
            ti = g / a.n_snr;
        }
        const uint64_t t = a.first_trial + (uint64_t)ti;
        const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32), qs = (uint32_t)(a.q_base + q);
        const float sigma = a.sigma[q];
        const bool first_item = g == 0;
        // ---- capture window (OFDM.c:945-955) + AWGN ----
        int rx_start = a.fixed_start;
        if (rx_start < 0) {
            const uint4 o = philox10(t_lo, t_hi, 0u, STREAM_START | qs, a.k0, a.k1);
            rx_start = (int)(o.x % (uint32_t)(a.wave_len - L));
        }
        float2 *r = rbase + (rx_start & 3);             // r[n] = capture sample n
        if (a.ext && first_item) {
            for (int n = tid; n < L; n += SYNC_THREADS) r[n] = a.ext[n];
        } else {
            const int b0 = rx_start >> 2, b1 = (rx_start + L - 1) >> 2;
            const PhiloxHead hd = philox_head(t_lo, t_hi, STREAM_NOISE | qs, a.k1);   // shared by all blocks
            const float Ksig = noise_k(sigma);
            // Gaussian k of the trial's stream goes to waveform sample k (as if Transmission_Over_Air
            // had drawn the whole waveform); only the captured samples are ever evaluated.
            // FRAME_CAP_U Philox blocks per lane per pass, their waveform loads issued first.
#ifndef FRAME_CAP_U
#define FRAME_CAP_U 3   // Philox blocks per lane per pass: 752-block captures in 2 full passes (A/B: +1.7 % over 4)
#endif
            // The waveform is FR_REPS copies of one filtered frame (OFDM.c:607-612): sample k is sample
            // k mod nfilt of the first copy, so every trial reads the same 7.8 KB (L1-resident) instead of
            // its own 24 KB window of the 78 KB waveform.  bm = the block's index within the copy
            // (nfilt is a multiple of 4; pb > SYNC_THREADS, so one conditional subtract per step).
            const uint32_t pb = (uint32_t)(a.wave_len / (4 * FR_REPS)), nb_wave = (uint32_t)(a.wave_len / 4);
            uint32_t bm = (uint32_t)(b0 + tid) % pb;
            for (int bb = b0 + tid; bb <= b1; bb += FRAME_CAP_U * SYNC_THREADS) {
                float2 v[FRAME_CAP_U][4];
#pragma unroll
                for (int u = 0; u < FRAME_CAP_U; ++u) {
                    const int b = bb + SYNC_THREADS * u;
#ifdef OFDM_FRAME_WAVE_FULL     // A/B: read the full 78 KB waveform
                    const float4 *s4 = reinterpret_cast<const float4 *>(a.wave + 4 * b);
#else
                    const float4 *s4 = reinterpret_cast<const float4 *>(a.wave + 4 * bm);
#endif
                    const bool in = b <= b1 && (uint32_t)b < nb_wave;
                    const float4 lo = in ? s4[0] : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 hi = in ? s4[1] : make_float4(0.f, 0.f, 0.f, 0.f);
                    v[u][0] = make_float2(lo.x, lo.y); v[u][1] = make_float2(lo.z, lo.w);
                    v[u][2] = make_float2(hi.x, hi.y); v[u][3] = make_float2(hi.z, hi.w);
                    bm = min(bm + SYNC_THREADS, bm + SYNC_THREADS - pb);     // (bm + 128) mod pb, unsigned
                }
#ifdef OFDM_FRAME_CAP_VKEYS   // A/B: the pass's Philox blocks together, round keys in VGPRs
                uint4 po[FRAME_CAP_U];
                if (a.noise == OFDM_NOISE_REAL) {
                    uint32_t c2s[FRAME_CAP_U];
#pragma unroll
                    for (int u = 0; u < FRAME_CAP_U; ++u) c2s[u] = (uint32_t)(bb + SYNC_THREADS * u);
                    philox10_c2_vk<FRAME_CAP_U>(hd, c2s, a.k0, a.k1, po);
                }
#endif
#pragma unroll
                for (int u = 0; u < FRAME_CAP_U; ++u) {
                    const int b = bb + SYNC_THREADS * u;
                    if (b > b1) break;
                    float2 w[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) w[j] = v[u][j];
                    if (a.noise == OFDM_NOISE_REAL) {   // real-only (D7): sigma z = sqrt(K log2 u1) (cos | sin)
#ifdef OFDM_FRAME_CAP_VKEYS
                        const Noise4 nz = noise4_of(po[u], Ksig);
#else
                        const Noise4 nz = noise4_of(philox10_c2(hd, (uint32_t)b, a.k0, a.k1), Ksig);
#endif
                        w[0].x = fmaf(nz.r0, nz.c0, w[0].x); w[1].x = fmaf(nz.r0, nz.s0, w[1].x);
                        w[2].x = fmaf(nz.r1, nz.c1, w[2].x); w[3].x = fmaf(nz.r1, nz.s1, w[3].x);
                    }
                    // samples of the block outside [0, L) land in the region's slack, never read as capture
                    float4 *d4 = reinterpret_cast<float4 *>(rbase + 4 * (b - b0));
                    d4[0] = make_float4(w[0].x, w[0].y, w[1].x, w[1].y);
                    d4[1] = make_float4(w[2].x, w[2].y, w[3].x, w[3].y);
                }
            }
        }
        for (int k = tid; k < cross_words(L); k += SYNC_THREADS) cross[k] = 0ull;
        __syncthreads();
#ifndef OFDM_FRAME_STATIC_ITEMS
        if (i + 1 < run_end) {
            inext = i + 1;
        } else {
            inext = (int64_t)__builtin_amdgcn_readfirstlane(redi[RED_I_NEXT]) * FRAME_ITEM_RUN;
            run_end = inext + FRAME_ITEM_RUN;
        }
#else
        inext = i + gridDim.x;
#endif
        FR_STAMP(0);                                           // capture + noise

        // ---- Word_Optimization_Analysis(Rx_filter_signal) (OFDM.c:38-73, 962-967): the full RRC
        // matched filter of the capture, min / max over real and imaginary parts (opt-in) ----
        if (a.word_stats) {
            float mn = 1e9f, mx = -1e9f;
            for (int k = tid; k < L + 20; k += SYNC_THREADS) {
                float2 v = make_float2(0.f, 0.f);
#pragma unroll
                for (int j = 0; j < 21; ++j) {
                    const int m = k - j;
                    if (m >= 0 && m < L) {
                        v.x = fmaf(r[m].x, a.taps[j], v.x);
                        v.y = fmaf(r[m].y, a.taps[j], v.y);
                    }
                }
                mn = fminf(mn, fminf(v.x, v.y));
                mx = fmaxf(mx, fmaxf(v.x, v.y));
            }
            mn = wave_min_f(mn);
            mx = wave_max_f(mx);
            __syncthreads();
            if (lane == 0) { redf[2 * (tid >> 6)] = mn; redf[2 * (tid >> 6) + 1] = mx; }
            __syncthreads();
            if (tid == 0) {
                float bmn = redf[0], bmx = redf[1];
                for (int w = 1; w < SYNC_WAVES; ++w) { bmn = fminf(bmn, redf[2 * w]); bmx = fmaxf(bmx, redf[2 * w + 1]); }
                unsigned long long *sl = acc + q * ACC_SLOTS;
                sl[10] = (unsigned long long)min((long long)sl[10], (long long)__float2ll_rn(bmn * (float)OFDM_EVM_Q_SCALE));
                sl[11] = (unsigned long long)max((long long)sl[11], (long long)__float2ll_rn(bmx * (float)OFDM_EVM_Q_SCALE));
            }
        }

        // ---- Packet_Detection (OFDM.c:659-683): M[n] = |sum r[n+k] r[n+k+16]|^2 / (sum |r[n+k+16]|^2)^2,
        // k < 32, no conjugate, on the UNFILTERED capture; sliding sums over each lane's chunk with the
        // LDS reads issued DET_B positions at a time.  M > 0.75 (OFDM.c:687, 695) is decided as the sign
        // of t = 0.75 den - num (fma: exact before its one rounding): t < 0 <=> crossing, which keeps the
        // division's outcomes 0/0 -> false (t = +0) and x/0 -> true (t = -num). ----
        const int n0 = tid * chunk, n1 = min(n0 + chunk, Lc);
        unsigned long long cmask = 0ull;            // crossing n at bit n - n0 (chunk <= 64)
#ifndef FRAME_DET_B
#define FRAME_DET_B 5
#endif
        constexpr int DET_B = FRAME_DET_B;
        if (n0 < n1) {
#ifdef OFDM_FRAME_DET_OLD      // A/B: products formed, then added (9 VALU per window term, 24 per position)
            float sx = 0.f, sy = 0.f, pw = 0.f;
#pragma unroll 8
            for (int k = 0; k < 32; ++k) {
                const float2 u = r[n0 + k], v = r[n0 + k + 16];
                sx += u.x * v.x - u.y * v.y;
                sy += u.x * v.y + u.y * v.x;
                pw += v.x * v.x + v.y * v.y;
            }
            for (int nb = n0; nb < n1; nb += DET_B) {
                float2 o0[DET_B], o1[DET_B], i0[DET_B], i1[DET_B];
#pragma unroll
                for (int k = 0; k < DET_B; ++k) {
                    o0[k] = r[nb + k]; o1[k] = r[nb + k + 16]; i0[k] = r[nb + k + 32]; i1[k] = r[nb + k + 48];
                }
                uint32_t m = 0u;
#pragma unroll
                for (int k = 0; k < DET_B; ++k) {
                    const float num = sx * sx + sy * sy, den = pw * pw;
                    m |= num > 0.75f * den ? 1u << k : 0u;
                    sx += (i0[k].x * i1[k].x - i0[k].y * i1[k].y) - (o0[k].x * o1[k].x - o0[k].y * o1[k].y);
                    sy += (i0[k].x * i1[k].y + i0[k].y * i1[k].x) - (o0[k].x * o1[k].y + o0[k].y * o1[k].x);
                    pw += (i1[k].x * i1[k].x + i1[k].y * i1[k].y) - (o1[k].x * o1[k].x + o1[k].y * o1[k].y);
                }
                cmask |= (unsigned long long)m << (nb - n0);
            }
#else
            // every window term accumulated by fma straight into the running sums (6 VALU per term; the
            // sliding update is 12 fma per position: the entering product added, the leaving one taken off)
            float sx = 0.f, sy = 0.f, pw = 0.f;
#pragma unroll 8
            for (int k = 0; k < 32; ++k) {
                const float2 u = r[n0 + k], v = r[n0 + k + 16];
                sx = fmaf(u.x, v.x, sx); sx = fmaf(-u.y, v.y, sx);
                sy = fmaf(u.x, v.y, sy); sy = fmaf(u.y, v.x, sy);
                pw = fmaf(v.x, v.x, pw); pw = fmaf(v.y, v.y, pw);
            }
            // t's sign bits shifted in with v_alignbit, one per position (first position highest); every
            // active lane runs the same ceil(chunk / DET_B) batches, positions past n1 are masked below
            uint32_t mlo = 0u, mhi = 0u;
            const int nbat = (chunk + DET_B - 1) / DET_B;
            for (int b = 0; b < nbat; ++b) {
                const int nb = n0 + DET_B * b;
                float2 o0[DET_B], o1[DET_B], i0[DET_B], i1[DET_B];
#pragma unroll
                for (int k = 0; k < DET_B; ++k) {       // reads past the capture land in the region's slack / cross
                    o0[k] = r[nb + k]; o1[k] = r[nb + k + 16]; i0[k] = r[nb + k + 32]; i1[k] = r[nb + k + 48];
                }
#pragma unroll
                for (int k = 0; k < DET_B; ++k) {
                    const float num = fmaf(sx, sx, sy * sy), h = 0.75f * pw;
                    const float t = fmaf(h, pw, -num);
                    if (chunk > 32) mhi = __builtin_amdgcn_alignbit(mhi, mlo, 31);
                    mlo = __builtin_amdgcn_alignbit(mlo, __float_as_uint(t), 31);
                    sx = fmaf(i0[k].x, i1[k].x, sx); sx = fmaf(-i0[k].y, i1[k].y, sx);
                    sx = fmaf(-o0[k].x, o1[k].x, sx); sx = fmaf(o0[k].y, o1[k].y, sx);
                    sy = fmaf(i0[k].x, i1[k].y, sy); sy = fmaf(i0[k].y, i1[k].x, sy);
                    sy = fmaf(-o0[k].x, o1[k].y, sy); sy = fmaf(-o0[k].y, o1[k].x, sy);
                    pw = fmaf(i1[k].x, i1[k].x, pw); pw = fmaf(i1[k].y, i1[k].y, pw);
                    pw = fmaf(-o1[k].x, o1[k].x, pw); pw = fmaf(-o1[k].y, o1[k].y, pw);
                }
            }
            // J = nbat * DET_B positions: position j sits at bit J - 1 - j of (mhi:mlo); reverse the bits
            const int J = nbat * DET_B;
            const unsigned long long rev = ((unsigned long long)__builtin_bitreverse32(mlo) << 32) |
                                           __builtin_bitreverse32(mhi);
            cmask = rev >> (64 - J);
#endif
            if (n1 - n0 < 64) cmask &= (1ull << (n1 - n0)) - 1ull;   // the last batch's positions past n1
            if (cmask) {
                atomicOr(&cross[n0 >> 6], cmask << (n0 & 63));
                if ((n0 & 63) + chunk > 64) atomicOr(&cross[(n0 >> 6) + 1], cmask >> (64 - (n0 & 63)));
            }
        }
        // first / last crossing in this lane's chunk
        const int first = cmask ? n0 + __builtin_ctzll(cmask) : -1;
        const int last = cmask ? n0 + 63 - __builtin_clzll(cmask) : -1;
        if (a.dbg_corr && first_item) {             // Corr_Out for ofdm_receiver's parity dump
            for (int n = tid; n < Lc; n += SYNC_THREADS) {
                float sx = 0.f, sy = 0.f, pw = 0.f;
                for (int k = 0; k < 32; ++k) {
                    const float2 u = r[n + k], v = r[n + k + 16];
                    sx += u.x * v.x - u.y * v.y;
                    sy += u.x * v.y + u.y * v.x;
                    pw += v.x * v.x + v.y * v.y;
                }
                a.dbg_corr[n] = (sx * sx + sy * sy) / (pw * pw);
            }
        }

        // ---- Packet_Selection (OFDM.c:685-771): crossing idx[j] is a front iff idx[j] - idx[j-1] > 300
        // (idx[-1] = -1).  Fronts are > 300 apart and a chunk is < 300 positions, so only a lane's
        // first crossing can be one, and its predecessor is the last crossing of the earlier chunks:
        // an exclusive prefix max over the block's lanes.  The first front x with a later front and
        // M[front+230] > 0.75 gives packet_idx = front + len_RRC_rx + 1; otherwise 0 (OFDM.c:752-761). ----
#ifdef OFDM_FRAME_SCAN_SHFL     // A/B: the ds_bpermute ladder
        int pm = last;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t2 = __shfl_up(pm, o, 64);
            if (lane >= o) pm = max(pm, t2);
        }
        int prev = __shfl_up(pm, 1, 64);
        if (lane == 0) prev = -1;
#else
        const int pm = wave_prefix_max(last);
        int prev = wave_shr1(pm);
#endif
        if (lane == 63) redi[RED_I_PREFIX + (tid >> 6)] = pm;   // each wave's last crossing
        __syncthreads();                            // crossing words and wave prefixes are in LDS
        for (int w = 0; w < (tid >> 6); ++w) prev = max(prev, redi[RED_I_PREFIX + w]);   // earlier waves
        const int front = (first >= 0 && first - prev > 300) ? first : -1;
        FR_STAMP(1);                                           // packet detection
        const bool valid = front >= 0 && front + 230 < Lc && bit_at(cross, front + 230);
        // the first valid front that has a later front: the least valid front, unless it is the last one
#ifdef OFDM_FRAME_MINMAX_LEAD   // A/B: the leading barrier kept
        const int2 mm = block_minmax_i<true>(valid ? front : 0x7fffffff, front, redi + RED_I_MINMAX);
#else
        const int2 mm = block_minmax_i<false>(valid ? front : 0x7fffffff, front, redi + RED_I_MINMAX);
#endif
        const int cand = mm.x < mm.y ? mm.x : 0x7fffffff;
        const bool sync_fail = cand == 0x7fffffff;
        const int p = sync_fail ? 0 : cand + 10 + 1;           // len_RRC_rx + 1 (OFDM.c:758)
        FR_STAMP(2);                                           // packet selection

        // fr[] in the unread prefix [0, off + lo) or suffix (off + hi, region) of the capture region
        if (a.fr_in_cap) {
            const int off = rx_start & 3, lo = max(p - 20, 0), hi = min(p + 2 * nfr - 2, L - 1);
            fr = off + lo >= nfr ? rbase : rbase + off + hi + 1;
        }
        // ---- RRC matched filter at the down-sampled instants p + 2i (OFDM.c:965, 992-996): outputs
        // interleaved over the lanes, so a tap's reads are 2 samples apart across lanes; clamped reads +
        // select are Convolution's zero padding.  Only the 160 + 64 nd frame samples the receiver reads
        // are filtered (needed_k: the coarse-CFO STF lag window, both LTFs, the data windows without
        // their CPs), all nfr for the single-capture dump.  The OOB flag is unchanged: the reference
        // reads past its buffer iff the last instant does, and the last sample is always needed. ----
        const bool dbg = a.dbg_frame && first_item;
        bool oob_l = false;
        // taps copied to VGPRs: an FMA with an SGPR operand issues in the slow class (+0.6 %)
        float tv[21];
#ifdef FRAME_TAPS_SGPR
#pragma unroll
        for (int j = 0; j < 21; ++j) tv[j] = a.taps[j];
#else
        {
            // read from the kernarg segment through a pointer made opaque per item, so the 21 taps are
            // scalar-loaded here and die at the copy instead of being hoisted into SGPRs held across the
            // item loop (they were most of the loop's SGPR spills)
            using kchar = __attribute__((address_space(4))) char;
            using kfloat = __attribute__((address_space(4))) float;
            const kfloat *tp = (const kfloat *)((const kchar *)__builtin_amdgcn_kernarg_segment_ptr() +
                                                    offsetof(FrameArgs, taps));
            asm volatile("" : "+s"(tp));
#pragma unroll
            for (int j = 0; j < 21; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(tv[j]) : "s"(tp[j]));
        }
#endif
#ifdef OFDM_FRAME_MF_ALL      // A/B: filter every frame sample
        const int nmf = nfr;
#else
        const int nmf = dbg ? nfr : 160 + 64 * a.n_data;
#endif
        for (int j = tid; j < nmf; j += SYNC_THREADS) {
#ifdef OFDM_FRAME_MF_ALL
            const int ii = j;
#else
            const int ii = dbg ? j : needed_k(j);
#endif
            const int n = p + 2 * ii;
            float2 v = make_float2(0.f, 0.f);
            if (n >= 20 && n < L) {                              // all 21 taps inside the capture
#ifdef OFDM_FRAME_MF_B64      // A/B: one ds_read_b64 per tap (lanes 16 B apart: 2-way bank conflicts)
                float2 x[21];
#pragma unroll
                for (int t = 0; t < 21; ++t) x[t] = r[n - t];
#else
                // samples n-20 .. n as 10 sample pairs + 1 single: a ds_read_b128 per pair, 16-byte
                // aligned in the region (rbase); lanes read adjacent 16 B (conflict-free).  The pairs start
                // at n-20 or n-19 depending on the parity of the region index, uniform per item.
                float2 x[21];                                    // x[t] = sample n - t
                const int s0 = n - 20 + (rx_start & 3);          // region index of sample n - 20
                auto load = [&](auto oc) {
                    constexpr int ODD = decltype(oc)::value;
                    const float4 *q4 = reinterpret_cast<const float4 *>(rbase + s0 + ODD);
#pragma unroll
                    for (int m = 0; m < 10; ++m) {
                        const float4 w = q4[m];                  // samples n-20+ODD+2m, n-19+ODD+2m
                        x[20 - ODD - 2 * m] = make_float2(w.x, w.y);
                        x[19 - ODD - 2 * m] = make_float2(w.z, w.w);
                    }
                    x[ODD ? 20 : 0] = rbase[ODD ? s0 : s0 + 20];  // the sample the pairs leave out
                };
                if (s0 & 1) load(std::integral_constant<int, 1>{});
                else load(std::integral_constant<int, 0>{});
#endif
#pragma unroll
                for (int t = 0; t < 21; ++t) {
                    v.x = fmaf(x[t].x, tv[t], v.x);
                    v.y = fmaf(x[t].y, tv[t], v.y);
                }
            } else if (n >= L + 20) {
                oob_l = true;                                    // the reference reads past its buffer
            } else {
#pragma unroll
                for (int t = 0; t < 21; ++t) {
                    const int m = n - t;
                    float2 x = r[min(max(m, 0), L - 1)];
                    x = (m >= 0 && m < L) ? x : make_float2(0.f, 0.f);
                    v.x = fmaf(x.x, tv[t], v.x);
                    v.y = fmaf(x.y, tv[t], v.y);
                }
            }
            fr[ii] = v;                                          // outside every lane's reads
        }
        // each wave's OOB flag, read by thread 0 after the barrier that also orders fr[] for every lane
        if (lane == 0) redi[RED_I_MAX + (tid >> 6)] = __ballot(oob_l) != 0ull;
        __syncthreads();
        FR_STAMP(3);                                           // matched filter + down-sample

        // ---- Coarse CFO (OFDM.c:773-804): 16-lag autocorrelation of the short preamble; fine CFO
        // (OFDM.c:806-828): 64-lag over the two long training symbols after the coarse rotation, the 128
        // rotated LTF samples formed on the fly (the same arithmetic as rotating the whole frame first).
        // Wave 0 holds every term: both estimates are wave reductions there, and one barrier hands the
        // frequencies to the other waves. ----
        double *cfo_sh = reinterpret_cast<double *>(redf);      // [fc, ff]
        if (tid < 64) {
            float2 pp = make_float2(0.f, 0.f);
            if (tid < 16) {
                const float2 u = fr[80 + tid], v = fr[96 + tid];
                pp = make_float2(u.x * v.x + u.y * v.y, u.y * v.x - u.x * v.y);
            }
            pp.x = wave_sum_f(pp.x);
            pp.y = wave_sum_f(pp.y);
            double fc = (-1.0 / (2.0 * M_PI * 16.0 * TS)) * (double)atan2f(pp.y, pp.x);
            if (a.float_cfo) fc = (double)(float)fc;
            const float2 u = cfo_rot(fr[192 + tid], fc * TS, 192 + tid), v = cfo_rot(fr[256 + tid], fc * TS, 256 + tid);
            pp = make_float2(u.x * v.x + u.y * v.y, u.y * v.x - u.x * v.y);
            pp.x = wave_sum_f(pp.x);
            pp.y = wave_sum_f(pp.y);
            double ff = (-1.0 / (2.0 * M_PI * 64.0 * TS)) * (double)atan2f(pp.y, pp.x);
            if (a.float_cfo) ff = (double)(float)ff;
            if (tid == 0) { cfo_sh[0] = fc; cfo_sh[1] = ff; }
        }
        __syncthreads();
        const double fc = cfo_sh[0], ff = cfo_sh[1];
        (void)fc; (void)ff;
        // ---- coarse then fine rotation (OFDM.c:802, 825) as ONE rotation by the summed phase
        // 2 pi (fc + ff) Ts k, evaluated in fp64 revolutions (the reference's two double-precision
        // cexp products rounded to float twice; the same rotation to fp32 rounding), the result handed
        // off directly: LTF1 [192,256), LTF2 [256,320), data d [336 + 80 d, +64) (OFDM.c:830-850,
        // 1024-1040) ----
        const int nw = 2 + a.n_data;
        float2 *dst = win_item(a.win, a.ipb, nw, i);
        const int row = a.ipb * nw;                            // float2 between samples n and n + 1
#ifndef OFDM_FRAME_CFO_TWO_STEP
        const double fcf_ts = (fc + ff) * TS;
#endif
        // hand-off element j = sample j / nw of window j % nw: consecutive lanes fill the item's nw
        // adjacent slots of a tile row (j / nw by a 16-bit reciprocal, exact for j < 64 nw <= 640);
        // the dump rotates all nfr samples
        const int nrot = dbg ? nfr : 64 * nw;
        const uint32_t inv_nw = (65536u + (uint32_t)nw - 1u) / (uint32_t)nw;
        for (int j = tid; j < nrot; j += SYNC_THREADS) {
            int n = (int)(((uint32_t)j * inv_nw) >> 16), w = j - n * nw;
            int k = needed_k(64 * w + n + 32);
            if (dbg) {
                k = j; w = -1;
                if (k >= 192 && k < 320) {
                    w = (k - 192) >> 6; n = (k - 192) & 63;
                } else if (k >= 336) {
                    const int d = (k - 336) / 80, o = k - 336 - 80 * d;
                    if (d < a.n_data && o < 64) { w = 2 + d; n = o; }
                }
            }
#ifdef OFDM_FRAME_CFO_TWO_STEP
            const float2 v = cfo_rot(cfo_rot(fr[k], fc * TS, k), ff * TS, k);
#else
            const float2 v = cfo_rot(fr[k], fcf_ts, k);
#endif
            if (dbg) a.dbg_frame[k] = v;
            if (w >= 0) dst[n * row + w] = v;
        }
        FR_STAMP(4);                                           // coarse + fine CFO + hand-off
        if (tid == 0) {
            int oob = 0;
#pragma unroll
            for (int w = 0; w < SYNC_WAVES; ++w) oob |= redi[RED_I_MAX + w];
            a.info[i] = make_int4(p, sync_fail, oob, rx_start);
            unsigned long long *sl = acc + q * ACC_SLOTS;
            sl[3] += sync_fail;
            sl[4] += oob;
            if (a.pidx_out) a.pidx_out[(int64_t)q * a.n_trials + ti] = p;
            if (first_item && a.dbg_ints) { a.dbg_ints[0] = p; a.dbg_ints[1] = sync_fail; a.dbg_ints[2] = oob; a.dbg_ints[3] = rx_start; }
        }
        __syncthreads();
        FR_STAMP(6);                                           // hand-off
    }
#ifdef OFDM_FRAME_STAMPS
    if (threadIdx.x == 0 && a.stamps)
        for (int k = 0; k < 7; ++k) atomicAdd(&a.stamps[k], stamp_acc[k]);
#endif
    __syncthreads();
    for (int k = tid; k < a.n_snr; k += SYNC_THREADS) {
        unsigned long long *c = a.counters + k * OFDM_NCOUNTERS;
        const unsigned long long *sl = acc + k * ACC_SLOTS;
        if (sl[3]) atomicAdd(&c[OFDM_C_SYNC_FAIL], sl[3]);
        if (sl[4]) atomicAdd(&c[OFDM_C_OOB], sl[4]);
        if (a.word_stats) {
            atomicMin(reinterpret_cast<long long *>(&c[OFDM_C_WL_MIN_Q]), (long long)sl[10]);
            atomicMax(reinterpret_cast<long long *>(&c[OFDM_C_WL_MAX_Q]), (long long)sl[11]);
        }
    }
}

// ---------------------------------------------------------------- K4b': symbols of the synced frames
// LS estimate + CP strip + fft + ZF + slicer + demap (OFDM.c:830-1165) for a batch of items: a quad
// carries {LTF1, LTF2, D_2k, D_2k+1} of one item (estimate formed inside the quad with two DPP
// broadcasts), ceil(n_data / 2) quads per item, 16 quads per wave.
constexpr int SYM_THREADS = 256;
template <bool DUMP>   // DUMP: item 0's bits / subcarriers / metrics for ofdm_receiver
#ifndef FRAME_SYM_MINB
#define FRAME_SYM_MINB 2   // 3 waves/SIMD spills 196 VGPRs: frame mode 9 % slower
#endif
__global__ __launch_bounds__(SYM_THREADS, FRAME_SYM_MINB) void frame_sym_kernel(FrameArgs a) {
    __shared__ unsigned long long acc[OFDM_MAX_SNR][8];
    __shared__ float part_e[SYM_THREADS / 4][2];             // per quad: EVM of its two data symbols
    __shared__ uint32_t part_b[SYM_THREADS / 4][2], part_a[SYM_THREADS / 4][2];
    for (int k = threadIdx.x; k < a.n_snr * 8; k += SYM_THREADS) (&acc[0][0])[k] = 0ull;
    __syncthreads();
    const int lane = threadIdx.x & 63, quad = threadIdx.x >> 2, role = lane & 3;
    const int qpi = (a.n_data + 1) / 2, ipb = (SYM_THREADS / 4) / qpi;   // quads per item, items per block
    const int item_l = quad / qpi, qi = quad - item_l * qpi;
    const int dsym = 2 * qi + (role & 1);
    const int nw = 2 + a.n_data;
    const int dsc = min(dsym, a.n_data - 1);
    const int w = role < 2 ? role : 2 + dsc;
    for (int64_t base = (int64_t)blockIdx.x * ipb; base < a.n_items; base += (int64_t)gridDim.x * ipb) {
        const int64_t i = base + item_l;
        const bool item_ok = item_l < ipb && i < a.n_items;
        const bool dlane = item_ok && role >= 2 && dsym < a.n_data;
        const float2 *src = win_item(a.win, ipb, nw, item_ok ? i : base) + w;
        const int row = ipb * nw;                                  // float2 between samples n and n + 1
        float2 x[64];
        // load fused with the first radix-4 stage, 16 samples at a time (fft() = DFT(x (-1)^n))
        static_for<0, 4>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            gcf2 *sp = (gcf2 *)src;
            opaque(sp);
            static_for<0, 16>([&](auto pc) {
                constexpr int n = 16 * (decltype(pc)::value >> 2) + 4 * g + (decltype(pc)::value & 3);
                const float2 v = gld(sp, n * row);
                x[n] = (n & 1) ? make_float2(-v.x, -v.y) : v;
            });
            static_for<0, 4>([&](auto ic) { dif_stage1<false, 4 * g + decltype(ic)::value>(x); });
            sched_fence();
        });
        const uint32_t wd[4] = {a.dtable[4 * dsc], a.dtable[4 * dsc + 1], a.dtable[4 * dsc + 2], a.dtable[4 * dsc + 3]};
        SymState st;
        sym_init(st);
        const bool dump = DUMP && a.dbg_eq && item_ok && a.item0 + i == 0 && dlane;
        float2 *deq = dump ? a.dbg_eq + 48 * dsym : nullptr;
        auto Hof = [&](float2 Y, auto binc) { return ls_equalise<decltype(binc)::value>(Y); };
        static_for<0, 4>([&](auto rc) {
            constexpr int R = decltype(rc)::value;
            dif_sub16<false, R>(x);
            demap_sub<DUMP, R, 2>(x, wd[R], Hof, deq, st);
            sched_fence();
        });
        if (role >= 2) {
            part_e[quad][role & 1] = dlane ? finish_evm<2>(st) : 0.f;
            part_b[quad][role & 1] = dlane ? st.be : 0u;
            part_a[quad][role & 1] = dlane ? st.ax : 0u;
        }
        if (DUMP && dump && a.dbg_bits) { a.dbg_bits[3 * dsym] = st.d[0]; a.dbg_bits[3 * dsym + 1] = st.d[1]; a.dbg_bits[3 * dsym + 2] = st.d[2]; }
        __syncthreads();
        if (item_ok && qi == 0 && role == 0) {
            // the item's totals in symbol order (deterministic), then the trial's metrics
            float fe = 0.f;
            uint32_t ferr = 0u, fax = 0u;
            for (int k = 0; k < qpi; ++k)
                for (int r2 = 0; r2 < 2; ++r2) {
                    fe += part_e[quad + k][r2]; ferr += part_b[quad + k][r2]; fax += part_a[quad + k][r2];
                }
            const int64_t g = a.item0 + i;
            const int q = (int)(g % a.n_snr);
            unsigned long long *sl = acc[q];
            atomicAdd(&sl[0], (unsigned long long)ferr);
            atomicAdd(&sl[1], (unsigned long long)(ferr > 0u));
            atomicAdd(&sl[2], (unsigned long long)fax);
            const float N = 48.0f * (float)a.n_data;
            atomicAdd(&sl[5], (unsigned long long)(int64_t)__float2ll_rn(fe * (float)OFDM_EVM_Q_SCALE));
            const float db = fe > 0.f ? fmaxf(3.01029995663981195214f * __builtin_amdgcn_logf(fe / N), -400.f) : -400.f;
            atomicAdd(&sl[6], (unsigned long long)(int64_t)__float2ll_rn(db * (float)OFDM_EVM_Q_SCALE));
            float dbp = -INFINITY;
            if (fax > 0u) {
                dbp = 3.01029995663981195214f * __builtin_amdgcn_logf(2.0f * (float)fax / N);
                atomicAdd(&sl[7], (unsigned long long)(int64_t)__float2ll_rn(dbp * (float)OFDM_EVM_Q_SCALE));
                atomicAdd(&sl[4], 1ull);
            }
            if (DUMP && g == 0 && a.dbg_res) { a.dbg_res[0] = db; a.dbg_res[1] = dbp; a.dbg_res[2] = (float)ferr / (96.0f * a.n_data); }
        }
        __syncthreads();
    }
    for (int k = threadIdx.x; k < a.n_snr * 6; k += SYM_THREADS) {
        const int q = k / 6, s2 = k % 6;
        const int slot = s2 < 3 ? s2 : s2 + 1;           // 0 bit_err, 1 frame_err, 2 axis, 4 finite, 5 pre, 6 dbpre, 7 dbpost
        const unsigned long long v = acc[q][slot];
        if (!v) continue;
        const int c = slot == 0 ? OFDM_C_BIT_ERR : slot == 1 ? OFDM_C_FRAME_ERR : slot == 2 ? OFDM_C_EVM_POST_AXIS
                    : slot == 4 ? OFDM_C_EVMDB_POST_FINITE : slot == 5 ? OFDM_C_EVM_PRE_Q : OFDM_C_EVMDB_PRE_Q;
        atomicAdd(&a.counters[q * OFDM_NCOUNTERS + c], v);
    }
    for (int q = threadIdx.x; q < a.n_snr; q += SYM_THREADS)
        if (acc[q][7]) atomicAdd(&a.counters[q * OFDM_NCOUNTERS + OFDM_C_EVMDB_POST_Q], acc[q][7]);
    if (blockIdx.x == 0 && a.add_totals) {
        for (int q = threadIdx.x; q < a.n_snr; q += SYM_THREADS) {
            unsigned long long *c = a.counters + q * OFDM_NCOUNTERS;
            const unsigned long long nt = (unsigned long long)a.n_trials, nd = (unsigned long long)a.n_data;
            atomicAdd(&c[OFDM_C_FRAMES], nt);
            atomicAdd(&c[OFDM_C_SYMBOLS], nd * nt);
            atomicAdd(&c[OFDM_C_BITS], 96ull * nd * nt);
            atomicAdd(&c[OFDM_C_EVM_TERMS], 48ull * nd * nt);
        }
    }
}

// ======================================================================== host side
// rcosdesign(0.5, 10, 2, 'sqrt') (Tester.m:112; OFDM.c:32 holds the same values as floats)
static void rrc_taps(float out[21]) {
    const double beta = 0.5, sps = 2.0, pi = M_PI;
    double h[21], e = 0.0;
    for (int i = 0; i < 21; ++i) {
        const double t = (i - 10) / sps;
        double b;
        if (t == 0.0) b = -1.0 / (pi * sps) * (pi * (beta - 1) - 4 * beta);
        else if (std::fabs(std::fabs(4 * beta * t) - 1.0) < 1e-12)
            b = 1.0 / (2 * pi * sps) * (pi * (beta + 1) * std::sin(pi * (beta + 1) / (4 * beta)) -
                                        4 * beta * std::sin(pi * (beta - 1) / (4 * beta)) +
                                        pi * (beta - 1) * std::cos(pi * (beta - 1) / (4 * beta)));
        else
            b = -4 * beta / sps * (std::cos((1 + beta) * pi * t) + std::sin((1 - beta) * pi * t) / (4 * beta * t)) /
                (pi * ((4 * beta * t) * (4 * beta * t) - 1));
        h[i] = b;
        e += b * b;
    }
    for (int i = 0; i < 21; ++i) out[i] = (float)(h[i] / std::sqrt(e));
}

}  // namespace ofdm

using namespace ofdm;

#define HIPOK(expr)                                                                             \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return set_error(OFDM_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

static int ensure_wave(Ctx *c, int conv, int payload) {
    if (conv != OFDM_CONV_C && conv != OFDM_CONV_MATLAB) return set_error(OFDM_E_ARG, "bad conv %d", conv);
    if (payload != OFDM_PAYLOAD_MESSAGE && payload != OFDM_PAYLOAD_TESTER)
        return set_error(OFDM_E_ARG, "frame mode needs a fixed payload (MESSAGE or TESTER), got %d", payload);
    const int key = conv * 4 + payload;      // ofdm_set_message resets the key
    if (c->wave_key == key) return OFDM_OK;
    WaveArgs a{};
    a.n_data = payload_table(payload, c->message, a.table);
    const int len = wave_len_for(a.n_data);
    int rc = c->ensure(&c->d_wave, &c->cap_wave, (size_t)len * sizeof(float2) + 64);
    if (rc) return rc;
    a.wave = (float2 *)c->d_wave;
    a.power = (double *)((char *)c->d_wave + (size_t)len * sizeof(float2));
    rrc_taps(a.taps);
    a.stf_scale = (float)std::sqrt(13.0 / 6.0);
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_C>, dim3(1), dim3(256), 0, c->stream, a);
    else hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_MATLAB>, dim3(1), dim3(256), 0, c->stream, a);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(&c->wave_power, a.power, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    c->wave_key = key;
    c->wave_len = len;
    c->wave_frames = a.n_data;
    return OFDM_OK;
}

// capture length: opts->cap_len, or the reference's int(0.307 * len) when 0 (OFDM.c:945)
static int capture_len(const Ctx *c, const ofdm_rx_opts *o) { return o->cap_len ? o->cap_len : cap_len_for(c->wave_frames); }

static int check_opts(const Ctx *c, const ofdm_rx_opts *o) {
    if (!o) return set_error(OFDM_E_ARG, "opts is NULL");
    const int L = capture_len(c, o);
    if (L < 400 || L > CAP_ABS_MAX || L > c->wave_len)
        return set_error(OFDM_E_ARG, "cap_len %d must be in [400, min(%d, waveform %d)]", L, CAP_ABS_MAX, c->wave_len);
    if (o->fixed_start > c->wave_len - L) return set_error(OFDM_E_ARG, "fixed_start beyond the waveform");
    return OFDM_OK;
}

static void fill_frame_args(FrameArgs &a, Ctx *c, const ofdm_rx_opts *o, int noise, uint64_t seed, int payload) {
    a.wave = (const float2 *)c->d_wave;
    a.cap_len = capture_len(c, o);
    a.float_cfo = o->float_cfo;
    a.matlab = o->matlab_slicer;
    a.fixed_start = o->fixed_start;
    a.noise = noise;
    a.wave_len = c->wave_len;
    a.k0 = (uint32_t)seed;
    a.k1 = (uint32_t)(seed >> 32);
    a.n_data = payload_table(payload, c->message, a.table);
    for (int d = 0; d < a.n_data; ++d) demap_words(a.table + 3 * d, a.dtable + 4 * d);
    a.word_stats = o->word_stats ? 1 : 0;
    rrc_taps(a.taps);
}

// bits needed for the largest magnitude, as OFDM.c:56-64
static int32_t word_bits(double mn, double mx) {
    const float max_abs = (float)std::fmax(std::fabs(mn), std::fabs(mx));
    return max_abs < 1.0f ? 1 : (int32_t)std::ceil(std::log2((double)max_abs)) + 1;
}

static unsigned occupancy_grid(const void *kernel, int threads, size_t lds, int cus, int64_t blocks, int waves = 2) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 2;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)per_cu * cus * waves));
}

constexpr int64_t FRAME_CHUNK_ITEMS = int64_t(1) << 18;   // items per sync -> symbol hand-off (<= 1 GB)

// K4b then K4b' over a.n_items items starting at a.item0, through the context's hand-off buffer
static int run_frame_chunk(Ctx *c, FrameArgs &a) {
    const int nw = 2 + a.n_data;
    a.ipb = (SYM_THREADS / 4) / ((a.n_data + 1) / 2);
    const size_t wbytes = (size_t)((a.n_items + a.ipb - 1) / a.ipb) * a.ipb * nw * 64 * sizeof(float2);
    int rc = c->ensure(&c->d_scratch, &c->cap_scratch, wbytes + (size_t)a.n_items * sizeof(int4) + 256);
    if (rc) return rc;
    a.win = (float2 *)c->d_scratch;
    a.info = (int4 *)((char *)c->d_scratch + ((wbytes + 255) & ~size_t(255)));
    const size_t lds = frame_lds_bytes(a.cap_len, a.n_data, a.n_snr);
#ifdef OFDM_FR_SEPARATE
    a.fr_in_cap = 0;
#else
    a.fr_in_cap = fr_in_capture(a.cap_len, a.n_data);
#endif
    if (!c->d_work) HIPOK(hipMalloc(&c->d_work, 256));
    a.work = (unsigned long long *)c->d_work;
    HIPOK(hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
#ifndef OFDM_FRAME_SYNC_WAVES
#define OFDM_FRAME_SYNC_WAVES 2
#endif
    const int sync_waves = OFDM_FRAME_SYNC_WAVES;
    hipLaunchKernelGGL(frame_sync_kernel,
                       dim3(occupancy_grid(reinterpret_cast<const void *>(&frame_sync_kernel), SYNC_THREADS, lds,
                                           c->cus, a.n_items, sync_waves)),
                       dim3(SYNC_THREADS), lds, c->stream, a);
    const int ipb = (SYM_THREADS / 4) / ((a.n_data + 1) / 2);
    const bool dump = a.dbg_eq || a.dbg_bits || a.dbg_res;
    const void *k = dump ? reinterpret_cast<const void *>(&frame_sym_kernel<true>)
                         : reinterpret_cast<const void *>(&frame_sym_kernel<false>);
    const dim3 grid(occupancy_grid(k, SYM_THREADS, 0, c->cus, (a.n_items + ipb - 1) / ipb));
    if (dump) hipLaunchKernelGGL(frame_sym_kernel<true>, grid, dim3(SYM_THREADS), 0, c->stream, a);
    else hipLaunchKernelGGL(frame_sym_kernel<false>, grid, dim3(SYM_THREADS), 0, c->stream, a);
    HIPOK(hipGetLastError());
    return OFDM_OK;
}

extern "C" {

int ofdm_transmitter(ofdm_ctx *ctx, int conv, int payload, int float_taps, float *tx_out, int32_t max_complex,
                     int32_t *len_out) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    (void)float_taps;   // taps are fp32 on the GPU either way (OFDM.c:32 values)
    if (!c || !tx_out || !len_out) return set_error(OFDM_E_ARG, "bad transmitter arguments");
    HIPOK(hipSetDevice(c->device));
    int rc = ensure_wave(c, conv, payload);
    if (rc) return rc;
    if (max_complex < c->wave_len) return set_error(OFDM_E_ARG, "tx_out needs %d complex samples", c->wave_len);
    HIPOK(hipMemcpyAsync(tx_out, c->d_wave, (size_t)c->wave_len * sizeof(float2), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    *len_out = c->wave_len;
    return OFDM_OK;
}

int ofdm_transmission_over_air(ofdm_ctx *ctx, const float *tx, float *ota, int32_t len, double snr_db, uint64_t seed,
                               uint64_t trial, int32_t snr_index) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || !tx || !ota || len <= 0) return set_error(OFDM_E_ARG, "bad transmission_over_air arguments");
    HIPOK(hipSetDevice(c->device));
    const size_t bytes = (size_t)len * sizeof(float2);
    int rc = c->ensure(&c->d_scratch, &c->cap_scratch, 2 * bytes + 64);
    if (rc) return rc;
    float2 *dx = (float2 *)c->d_scratch, *dy = dx + len;
    double *dp = (double *)(dy + len);
    HIPOK(hipMemcpyAsync(dx, tx, bytes, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(power_kernel, dim3(1), dim3(256), 0, c->stream, (const float2 *)dx, (int)len, dp);
    const int nb = (len + 3) / 4;
    hipLaunchKernelGGL(ota_kernel, dim3((nb + 255) / 256), dim3(256), 0, c->stream, (const float2 *)dx, dy, (int)len,
                       (const double *)dp, std::pow(10.0, snr_db / 10.0), (uint32_t)trial, (uint32_t)(trial >> 32),
                       (uint32_t)snr_index, (uint32_t)seed, (uint32_t)(seed >> 32));
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(ota, dy, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    return OFDM_OK;
}

int ofdm_receiver(ofdm_ctx *ctx, const float *capture, const ofdm_rx_opts *opts, int payload, float *res3,
                  int32_t *ints4, int32_t *bits_out, float *eq_out) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || !capture) return set_error(OFDM_E_ARG, "bad receiver arguments");
    HIPOK(hipSetDevice(c->device));
    int rc = ensure_wave(c, OFDM_CONV_C, payload);
    if (rc) return rc;
    if ((rc = check_opts(c, opts))) return rc;
    const int L = capture_len(c, opts), nd = c->wave_frames;
    // scratch: capture | counters | res | ints | bits | eq
    const size_t off_cnt = ((size_t)L * sizeof(float2) + 255) & ~size_t(255);
    const size_t off_res = off_cnt + OFDM_NCOUNTERS * 8, off_int = off_res + 16, off_bits = off_int + 16;
    const size_t off_eq = off_bits + 4 * 3 * FR_MAX_DATA, total = off_eq + 48 * FR_MAX_DATA * sizeof(float2);
    if ((rc = c->ensure(&c->d_scratch2, &c->cap_scratch2, total))) return rc;
    char *base = (char *)c->d_scratch2;
    HIPOK(hipMemcpyAsync(base, capture, (size_t)L * sizeof(float2), hipMemcpyHostToDevice, c->stream));
    HIPOK(hipMemsetAsync(base + off_cnt, 0, total - off_cnt, c->stream));
    FrameArgs a{};
    fill_frame_args(a, c, opts, OFDM_NOISE_NONE, 0, payload);
    a.ext = (const float2 *)base;
    a.first_trial = 0;
    a.n_trials = 1;
    a.n_snr = 1;
    a.fixed_start = 0;
    a.counters = (unsigned long long *)(base + off_cnt);
    a.dbg_res = (float *)(base + off_res);
    a.dbg_ints = (int32_t *)(base + off_int);
    a.dbg_bits = (uint32_t *)(base + off_bits);
    a.dbg_eq = (float2 *)(base + off_eq);
    a.item0 = 0;
    a.n_items = 1;
    a.add_totals = 1;
    c->tic(Ctx::K_FRAME);
    rc = run_frame_chunk(c, a);
    c->toc();
    if (rc) return rc;
    float res[4];
    int32_t ints[4];
    uint32_t words[3 * FR_MAX_DATA];
    float2 eq[48 * FR_MAX_DATA];
    HIPOK(hipMemcpyAsync(res, base + off_res, 16, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(ints, base + off_int, 16, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(words, base + off_bits, sizeof(words), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(eq, base + off_eq, sizeof(eq), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    if (res3) { res3[0] = res[0]; res3[1] = res[1]; res3[2] = res[2]; }
    if (ints4) { ints4[0] = ints[0]; ints4[1] = ints[1]; ints4[2] = ints[2]; ints4[3] = nd; }
    if (bits_out)
        for (int b = 0; b < 96 * nd; ++b) bits_out[b] = (int32_t)((words[b / 32] >> (31 - (b & 31))) & 1u);
    if (eq_out) std::memcpy(eq_out, eq, (size_t)48 * nd * sizeof(float2));
    return OFDM_OK;
}

int ofdm_frame_sweep(ofdm_ctx *ctx, const ofdm_cfg *cfg, const ofdm_rx_opts *opts, const double *snr_db, int n_snr,
                     uint64_t first_trial, int64_t n_trials, int64_t *counters, int32_t *packet_idx) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (!opts) return set_error(OFDM_E_ARG, "opts is NULL");
    if (n_snr < 0 || (n_snr && (!snr_db || !counters)) || n_trials < 0) return set_error(OFDM_E_ARG, "bad sweep args");
    if (cfg->channel != OFDM_CHAN_AWGN) return set_error(OFDM_E_ARG, "frame mode models the AWGN channel only");
    if (cfg->noise == OFDM_NOISE_COMPLEX) return set_error(OFDM_E_ARG, "frame mode noise is real (OFDM.c:651) or none");
    if (n_snr == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    if ((rc = ensure_wave(c, cfg->conv, cfg->payload))) return rc;
    if ((rc = check_opts(c, opts))) return rc;
    const size_t cbytes = (size_t)n_snr * OFDM_NCOUNTERS * 8;
    const size_t pbytes = packet_idx ? (size_t)n_snr * n_trials * 4 : 0;
    if ((rc = c->ensure(&c->d_cnt, &c->cap_cnt, cbytes + pbytes + 256))) return rc;
    std::vector<int64_t> init((size_t)n_snr * OFDM_NCOUNTERS, 0);
    if (opts->word_stats)
        for (int q = 0; q < n_snr; ++q) {
            init[(size_t)q * OFDM_NCOUNTERS + OFDM_C_WL_MIN_Q] = INT64_MAX;
            init[(size_t)q * OFDM_NCOUNTERS + OFDM_C_WL_MAX_Q] = INT64_MIN;
        }
    HIPOK(hipMemcpyAsync(c->d_cnt, init.data(), cbytes, hipMemcpyHostToDevice, c->stream));
    int32_t *dp = packet_idx ? (int32_t *)((char *)c->d_cnt + ((cbytes + 255) & ~size_t(255))) : nullptr;
    for (int q0 = 0; q0 < n_snr; q0 += OFDM_MAX_SNR) {
        FrameArgs a{};
        fill_frame_args(a, c, opts, cfg->noise, cfg->seed, cfg->payload);
        a.first_trial = first_trial;
        a.n_trials = n_trials;
        a.n_snr = std::min(OFDM_MAX_SNR, n_snr - q0);
        a.q_base = q0;
        a.counters = (unsigned long long *)c->d_cnt + (size_t)q0 * OFDM_NCOUNTERS;
        a.pidx_out = dp ? dp + (size_t)q0 * n_trials : nullptr;
        for (int q = 0; q < a.n_snr; ++q)   // sigma^2 = P / 10^(snr/10) (OFDM.c:645-647)
            a.sigma[q] = (float)std::sqrt(c->wave_power / std::pow(10.0, snr_db[q0 + q] / 10.0));
        if (n_trials == 0) continue;
#ifdef OFDM_FRAME_STAMPS
        unsigned long long *dst = nullptr;
        HIPOK(hipMalloc(&dst, 64));
        HIPOK(hipMemset(dst, 0, 64));
        a.stamps = dst;
#endif
        const int64_t items = n_trials * a.n_snr;
        c->tic(Ctx::K_FRAME);
        for (int64_t i0 = 0; i0 < items; i0 += FRAME_CHUNK_ITEMS) {
            a.item0 = i0;
            a.n_items = std::min(FRAME_CHUNK_ITEMS, items - i0);
            a.add_totals = i0 + a.n_items >= items;
            if ((rc = run_frame_chunk(c, a))) { c->toc(); return rc; }
        }
        c->toc();
#ifdef OFDM_FRAME_STAMPS
        unsigned long long hs[8];
        HIPOK(hipMemcpy(hs, dst, 64, hipMemcpyDeviceToHost));
        hipFree(dst);
        static const char *names[7] = {"capture+noise", "detection", "selection", "matched filter", "cfo", "-",
                                       "hand-off"};
        double tot = 0;
        for (int k = 0; k < 7; ++k) tot += (double)hs[k];
        for (int k = 0; k < 7; ++k)
            fprintf(stderr, "frame stamp %-15s %6.2f%%  %.0f cycles/item\n", names[k], 100.0 * hs[k] / tot,
                    (double)hs[k] / (double)(n_trials * a.n_snr));
#endif
    }
    HIPOK(hipMemcpyAsync(counters, c->d_cnt, cbytes, hipMemcpyDeviceToHost, c->stream));
    if (dp) HIPOK(hipMemcpyAsync(packet_idx, dp, pbytes, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    if (opts->word_stats && n_trials > 0)
        for (int q = 0; q < n_snr; ++q) {
            int64_t *row = counters + (size_t)q * OFDM_NCOUNTERS;
            row[OFDM_C_WL_BITS] = word_bits(row[OFDM_C_WL_MIN_Q] / OFDM_EVM_Q_SCALE, row[OFDM_C_WL_MAX_Q] / OFDM_EVM_Q_SCALE);
        }
    return OFDM_OK;
}

int ofdm_word_length_report(ofdm_ctx *ctx, const float *capture, int32_t cap_len, float *out3, int32_t *bits) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c || !capture || cap_len <= 0 || cap_len > (1 << 24)) return set_error(OFDM_E_ARG, "bad word-length arguments");
    HIPOK(hipSetDevice(c->device));
    const size_t bytes = (size_t)cap_len * sizeof(float2);
    int rc = c->ensure(&c->d_scratch2, &c->cap_scratch2, bytes + 64);
    if (rc) return rc;
    float2 *dx = (float2 *)c->d_scratch2;
    float *dout = (float *)((char *)c->d_scratch2 + bytes);
    HIPOK(hipMemcpyAsync(dx, capture, bytes, hipMemcpyHostToDevice, c->stream));
    FrameArgs a{};
    rrc_taps(a.taps);
    hipLaunchKernelGGL(word_length_kernel, dim3(1), dim3(256), 0, c->stream, (const float2 *)dx, (int)cap_len, a, dout);
    HIPOK(hipGetLastError());
    float mm[2];
    HIPOK(hipMemcpyAsync(mm, dout, sizeof(mm), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    const float max_abs = std::fmax(std::fabs(mm[0]), std::fabs(mm[1]));
    if (out3) { out3[0] = mm[0]; out3[1] = mm[1]; out3[2] = max_abs; }
    if (bits) *bits = word_bits(mm[0], mm[1]);
    return OFDM_OK;
}

}  // extern "C"
