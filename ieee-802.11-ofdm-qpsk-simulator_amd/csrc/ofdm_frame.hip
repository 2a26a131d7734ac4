// ofdm_frame.hip -- frame mode: the reference's own trial on gfx950.
//
//   K4a frame_wave_kernel : Transmitter() (OFDM.c:467-618) -- preambles + data symbols, 2x zero
//                           stuffing, 21-tap RRC, x10 repeat, mean power (OFDM.c:637-643).
//   K4b frame_sync_kernel : one wave per (trial, SNR) item: capture (OFDM.c:945-955) + real AWGN
//                           (OFDM.c:651) in LDS (real parts; the imaginary parts are the clean waveform's),
//                           Packet_Detection (659-683) as fma-chained sliding sums with sign-bit crossings,
//                           Packet_Selection (685-771) as a DPP prefix max + wave min/max, the RRC matched
//                           filter only at the down-sampled instants the receiver reads (965, 984-996),
//                           coarse/fine CFO (773-828) as wave reductions, and the rotated LTF / data
//                           windows handed to
//   K4b' frame_sym_kernel : the same register FFT + LS estimate + demap as symbol mode (830-1165).
//   K4c ota_kernel        : Transmission_Over_Air() on a caller-provided waveform.
//
// The capture's real parts live in LDS (12 KB per trial for the reference's 2-symbol message; frames carry
// 1..8 data symbols, ofdm_set_message); detection keeps only the >0.75 crossings as per-lane bit masks,
// since Packet_Selection needs nothing else (it re-reads Corr_Out only at front+230).
#include "ofdm_internal.h"
#include "ofdm_ctx.h"
#include "ofdm_rxcommon.h"
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

// ofdm_frame_sym.hip / ofdm_frame_fix.hip include this file to instantiate one kernel each in a translation unit of
// its own (their own scheduler flags, build_lib.SOURCE_FLAGS); everything else lives in this one
#if defined(OFDM_FRAME_SYM_TU) || defined(OFDM_FRAME_FIX_TU) || defined(OFDM_FRAME_LONG_TU)
#define OFDM_FRAME_AUX_TU 1
#endif

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
    int32_t no_lazy;                // 1: evaluate every capture in full (OFDM_FRAME_NO_LAZY, the lazy path's test)
    int32_t fr_in_cap;              // fr[] inside the capture region (fr_in_capture)
    int32_t imt_len, im_period;     // LDS table of the capture's imaginary parts: length, index period
    uint32_t im_magic;              // ceil(2^32 / im_period): x mod im_period by one multiply-high (x < 2^14)
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
    int32_t region_floats;          // LDS floats per wave (wave_region_floats)
    // item0 = trial0 n_snr + q0: chunk item i is trial trial0 + (q0 + i) / n_snr, SNR (q0 + i) % n_snr, a 32-bit
    // division by one multiply-high with snr_magic = floor((2^32 - 1) / n_snr) (snr_divmod; run_frame_chunk)
    int64_t trial0;
    int32_t q0;
    uint32_t snr_magic;
    const float *wave_re;           // real parts of one waveform copy (nfilt floats; ensure_wave), the capture's clean part
};

// x / d and x % d for 32-bit x and d >= 1: with m = floor((2^32 - 1) / d) >= (2^32 - d) / d,
// x / d - 1 < x / d - x / 2^32 <= x m / 2^32 <= x / d, so t = mulhi(x, m) is the quotient or one less and one
// correction step finishes it.  On wave-uniform operands it stays on the scalar unit (the compiler's udiv
// expansion goes through VALU float reciprocals, and was re-done per item)
__host__ __device__ __forceinline__ uint32_t snr_divmod(uint32_t x, uint32_t d, uint32_t magic, uint32_t &r) {
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t t = __umulhi(x, magic);
#else
    uint32_t t = (uint32_t)(((uint64_t)x * magic) >> 32);
#endif
    r = x - t * d;
    if (r >= d) {
        ++t;
        r -= d;
    }
    return t;
}

#ifdef OFDM_FRAME_STAMPS   // diagnostic build: s_memtime per phase, summed over the grid
#define FR_STAMP(k)                                                                  \
    do {                                                                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
        if (threadIdx.x == 0) stamp_acc[k] += t_ - stamp_t;                          \
        stamp_t = t_;                                                                \
    } while (0)
constexpr bool FRAME_STAMPS_BUILD = true;   // frame_sync_long_kernel has no stamps: long captures run generic
#else
#define FR_STAMP(k) do { } while (0)
constexpr bool FRAME_STAMPS_BUILD = false;
#endif

// ======================================================================== K4a: waveform
#ifndef OFDM_FRAME_AUX_TU
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
#endif

// ======================================================================== K4c: over the air
// Transmission_Over_Air (OFDM.c:635-655): P = mean|x|^2, sigma^2 = P/10^(snr/10), real-only noise
// (D7), Gaussian k of stream (seed, trial, snr_index).
#ifndef OFDM_FRAME_AUX_TU   // the non-template kernels live in this translation unit only
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
#endif

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
#ifndef OFDM_FRAME_AUX_TU
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
#endif

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

// Hand-off: nw = 1 + n_data windows per item -- the SUM of the two rotated long training symbols (the channel
// estimate only uses FFT(LTF1) + FFT(LTF2) = FFT(LTF1 + LTF2), OFDM.c:846-849, fft() being linear) and the n_data
// data windows -- in tiles of ipb items (one frame_sym_kernel block).  Sample n = 16 q + r of a window sits at
// position p = 4 r + q, and a tile holds [4 groups][ipb items][16 positions][nw windows] float2, so that
//   * group g holds samples {16 q + r : 4 g <= r < 4 g + 4, q < 4}: exactly the 16 samples the symbol kernel's
//     load pass g reads (its first radix-4 stage combines x[n], x[n + 16], x[n + 32], x[n + 48]), as one run of
//     16 nw slots (128 nw bytes, whole 128-B lines) per item;
//   * the sync wave that owns the item writes those whole lines (the round-3 [64 samples][ipb items][nw] tile
//     wrote 32-B fragments 2 KB apart, 2.03x write amplification).
constexpr int WIN_SG = 16;
// frame_sym_kernel quads per item: 2 data lanes per quad for 1..2 data symbols (the reference frame: one quad),
// 3 for longer messages (OFDM_FRAME_SYM_DPQ2=1: 2 always, the equivalence test)
inline int sym_quads(int n_data) {
    const int dpq = n_data <= 2 || getenv("OFDM_FRAME_SYM_DPQ2") ? 2 : 3;
    return (n_data + dpq - 1) / dpq;
}
__host__ __device__ inline float2 *win_item(float2 *win, int ipb, int nw, int64_t item) {
    const int64_t tile = item / ipb, it = item - tile * ipb;
    return win + tile * 64 * (int64_t)(ipb * nw) + it * (WIN_SG * nw);
}
// offset of sample n of window 0 from win_item()
__host__ __device__ inline int win_off(int n, int ipb, int nw) {
    const int p = ((n & 15) << 2) | (n >> 4);
    return (p / WIN_SG) * (ipb * WIN_SG * nw) + (p % WIN_SG) * nw;
}

// j-th frame sample the receiver reads (j < 160 + 64 nd): the coarse-CFO lag window [80, 112)
// (OFDM.c:786-792), LTF1 + LTF2 [192, 320) (809-815, 830-850), data symbol d's FFT window [336 + 80 d, +64)
__device__ __forceinline__ int needed_k(int j) {
    if (j < 32) return 80 + j;
    if (j < 160) return 160 + j;
    const int e = j - 160;
    return 336 + 80 * (e >> 6) + (e & 63);
}

// ---------------------------------------------------------------- K4b: sync (one WAVE per item)
// Every (trial, SNR) item is processed by one wave from capture to hand-off: packet detection, selection and
// both CFO estimates are wave reductions (DPP / readlane), so the item needs no block barrier at all.  A block
// of SYNC_WAVES waves only shares LDS: the imaginary parts of one waveform copy (the noise is real-only, D7:
// a capture's imaginary part IS the clean waveform's, so each wave stores only the real parts of its
// capture) and the per-SNR accumulators.  LDS per block (reference message): 4 x 12.1 KB captures + 4.4 KB
// table = 53 KB, three blocks = 12 waves (3 per SIMD) per CU.
#define FRAME_SYNC_WAVES 4
constexpr int SYM_THREADS = 256;    // frame_sym_kernel block: its items per block set the hand-off tile
constexpr size_t FRAME_LDS_PER_CU = 160 * 1024;
constexpr int SYNC_WAVES = FRAME_SYNC_WAVES;
constexpr int SYNC_THREADS = 64 * SYNC_WAVES;
// frame_sync_long_kernel's block: 12 waves, one block per CU (12 x 12,288 B of capture rings + one 15,952-B table +
// 256 B = 163,664 B of the CU's 163,840), at most 168 VGPRs: 3 waves on every SIMD.  Round 6 A/Bs: 4-wave blocks with
// two rounds resident (two blocks per CU, 2 waves per SIMD) 8.02-8.05e8; 9-wave blocks, two rounds resident, 3, 2, 2, 2
// waves per SIMD 8.37-8.40e8 (profiles/r06/frame/ab_long9.txt); 12-wave blocks, one round resident 8.58-8.62e8
// (ab_long12.txt); 12-wave blocks with the capture ring 8.76-8.78e8 (ab_ring.txt); every counter and packet_idx unchanged.
constexpr int LONG_W = 12;
#define FRAME_LONG_MINW 3
constexpr int IMT_EXT = 128;         // table slack past one waveform copy: a lane's longest contiguous read
// The fixed-geometry kernel's layout: FIX_W waves per block sharing FIX_IMT_COPIES consecutive
// copies of the imaginary-part period.  With one copy every lane reduces its own table index mod the period, and the
// lanes past the wrap land 12 banks off the others (2-way conflicts on every imaginary detection load); with enough
// copies a detection round or a matched-filter pass reduces ONE uniform base and its lanes read a linear run (no
// lane-dependent wrap).  Three copies cover round 0's 2,031 samples from any start; 12-wave blocks (one per CU, the
// same 3 waves per SIMD) pay the table once per CU: 256 + 12,272 + 12 x 12,080 B = 157.5 KB.  Round 6 A/B
// (profiles/r06/frame/ab_layouts.txt): LDS conflicts 35.7 -> 23.6 % of the sync kernel's LDS array cycles, frame
// +1.4 % (5.37 -> 5.45e8); 12-wave blocks with one copy alone +0.0 %, three copies at 4-wave blocks -15 % (two blocks
// per CU).
constexpr int FIX_W = 12, FIX_IMT_COPIES = 3;
// Bank-balanced round-1 chunk starts (DetGeom::r1_start_of): conflicts 23.6 -> 10.5 %, but 15 more VALU per item for
// the start / owner arithmetic and -0.6 % (profiles/r06/frame/ab_balanced_r1.txt): off
constexpr bool LDS_BALANCED_R1 = false;
constexpr int DET_B = 16;           // detection positions per batch (= samples per register block)
// detection positions per lane and round: the largest odd chunk whose ceil(chunk / DET_B) batches fit one
// 64-bit crossing mask (63 for DET_B = 16); at most 2 rounds
constexpr int det_max_chunk() {
    int c = 63;
    while ((c + DET_B - 1) / DET_B * DET_B > 64) c -= 2;
    return c;
}
constexpr int DET_MAX_CHUNK = det_max_chunk();
static_assert(64 * 2 * DET_MAX_CHUNK + 47 >= CAP_ABS_MAX, "two detection rounds cover every capture");
#define FRAME_ITEM_RUN 4            // items per hand-out of the sync kernel's work counter (per wave)
#define FRAME_LAZY 1        // lazy capture + detection (see frame_sync_kernel; A/B: +5.3 %, profiles/r03/ab_n/)
#define FRAME_R1_SPREAD 1   // round 1 in one 16-position batch where spread chunks allow (A/B option)
#define FRAME_LAZY_C0 31    // round-0 positions per lane when lazy (two 16-position batches)
// Detection geometry for Lc = cap_len - 47 positions: R rounds of 64 lanes, round 0 c0 positions per lane over
// [0, B1 = 64 c0), round 1 c1 per lane from B1 (chunks odd: the lanes' LDS reads fall in distinct banks)
struct DetGeom {
    int c0, c1, x1, B1, R;
    // first position of lane l's round-1 chunk, relative to B1
    __host__ __device__ int r1_start(int l) const { return r1_start_of(c1, x1, l); }
    // x1 of the 64 chunks are one position longer.  Spread evenly (l c1 + floor(l x1 / 64)), the starts of a 32-lane
    // half fall on 31 distinct banks mod 32, and every dword access of round 1 is 2-way; the reference capture's
    // (c1, x1) = (15, 17) has a layout whose starts are distinct mod 32 in each half (a search over the 16/15 chunk
    // sequences): 16-position chunks on lanes 8, 10, .., 22 of each half and on lane 31.  LDS_BALANCED_R1 selects
    // it; the crossing look-up's owner estimate is within one lane of it (every position checked on the host).
    __host__ __device__ static int r1_start_of(int c1, int x1, int l) {
        if (LDS_BALANCED_R1 && c1 == 15 && x1 == 17)
            return 15 * l + min(8, max(0, ((l & 31) - 7) >> 1)) + 9 * (l >> 5) - (l >> 6);
        return l * c1 + ((l * x1) >> 6);
    }
    __host__ __device__ static DetGeom of(int Lc) {
        DetGeom g{};
        // Lazy: round 0 covers the first 64 FRAME_LAZY_C0 positions (the reference capture: 1984 of 2961), and
        // only the capture samples round 0 reads are generated before it; when round 0 alone decides
        // Packet_Selection and the matched filter reads inside that part, the rest of the capture and round 1
        // are skipped (same packet_idx, same frame: see the selection in frame_sync_kernel).
        g.c0 = Lc > 64 * FRAME_LAZY_C0 ? FRAME_LAZY_C0 : (((Lc + 63) / 64) | 1);
        g.B1 = 64 * g.c0;
        g.R = Lc > g.B1 ? 2 : 1;
        // round 1: a uniform odd chunk, or -- when that saves a 16-position batch (the reference capture: 977
        // positions = 64 x 15 + 17, one batch instead of two of chunk 17) -- c1 positions per lane plus one more
        // on x1 lanes spread evenly (lane l starts at B1 + l c1 + floor(l x1 / 64): at most 2-way bank conflicts)
        g.c1 = g.R == 2 ? (((Lc - g.B1 + 63) / 64) | 1) : g.c0;
        g.x1 = 0;
        if (g.R == 2) {
            const int c1b = (Lc - g.B1) / 64, r1 = (Lc - g.B1) - 64 * c1b;
            if (FRAME_R1_SPREAD && (c1b + (r1 > 0) + DET_B - 1) / DET_B < (g.c1 + DET_B - 1) / DET_B) {
                g.c1 = c1b;
                g.x1 = r1;
            }
        }
        return g;
    }
    // the last capture sample (relative to the capture start) a detection round's register blocks load: every
    // active lane loads ceil(chunk / DET_B) + 3 blocks of DET_B from its first position, the last active lane's
    // reaching furthest (up to 3 blocks past the capture)
    __host__ __device__ int max_read(int Lc) const {
        int m = 0;
        const int nb0 = (c0 + DET_B - 1) / DET_B, l0 = min(63, (Lc - 1) / c0);
        m = max(m, l0 * c0 + DET_B * (nb0 + 3) - 1);
        if (R == 2) {
            const int nb1 = (c1 + (x1 > 0) + DET_B - 1) / DET_B;
            int l1 = 63;
            while (l1 > 0 && B1 + r1_start(l1) >= Lc) --l1;
            m = max(m, B1 + r1_start(l1) + DET_B * (nb1 + 3) - 1);
        }
        return m;
    }
};
// per-SNR block accumulators: sync failures, OOB reads (and, with word_stats, the word-length min / max)
__host__ __device__ inline int acc_slots(int word_stats) { return word_stats ? 4 : 2; }
// capture region (floats), a multiple of 4 (16-byte aligned regions): the capture starts at float (rx_start & 3)
// so that every Philox block of 4 samples is one 16-byte aligned ds_write_b128; the region holds the capture's
// L + 8 floats, the detection blocks the last active lane loads (DetGeom::max_read) and the matched-filter runs'
// last window (a run cut short at the end of a needed range reads up to L + 5, i.e. float L + 8)
__host__ __device__ inline int cap_region(int cap_len) {
    const int det = 3 + DetGeom::of(cap_len - 47).max_read(cap_len - 47) + 1;
    return (max(cap_len + 9, det) + 3) & ~3;
}
// The filtered frame fr[] (float2, indexed by frame sample) goes into the part of the capture region the
// matched filter does not read: it reads 2 nfr + 19 floats, so the unread prefix or suffix holds the 2 nfr
// floats of fr[] whenever the region has 6 nfr + 24.  Shorter user captures get fr[] after the region.
__host__ __device__ inline bool fr_in_capture(int cap_len, int n_data) {
    return cap_region(cap_len) >= 6 * fr_len(n_data) + 24;
}
__host__ __device__ inline int wave_region_floats(int cap_len, int n_data) {
    return cap_region(cap_len) + (fr_in_capture(cap_len, n_data) ? 0 : 2 * fr_len(n_data));
}
__host__ __device__ inline size_t frame_lds_bytes(int cap_len, int n_data, int n_snr, int imt_len, int word_stats,
                                                  int waves = SYNC_WAVES) {
    return (size_t)n_snr * acc_slots(word_stats) * 8 + (((size_t)imt_len * 4 + 15) & ~size_t(15)) +
           (size_t)waves * wave_region_floats(cap_len, n_data) * 4;
}

// LDS ordering between the lanes of one wave (no block barrier: the other waves run other items)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x mod the table period for 0 <= x < 2^14 (q = floor(x / period) by multiply-high: exact there)
struct ImMod {
    int period;
    uint32_t magic;      // ceil(2^32 / period)
    __device__ __forceinline__ int operator()(int x) const {
        const uint32_t q = __umulhi((uint32_t)x, magic);
        return x - (int)(q * (uint32_t)period);
    }
};

// N (odd) contiguous LDS floats x[k] = p[s + k] as (N - 1) / 2 ds_read_b64 + 1 ds_read_b32; ODD = s & 1 (uniform
// per item), so the pairs are 8-byte aligned
// The pairs are read through an 8-byte vector type in the LDS address space, so that each is one ds_read_b64
// (64 banks of 4 B, 2 LDS cycles per wave-instruction) and not a ds_read2_b32 (two 32-bank dword accesses, 4
// cycles): the matched filter's lane starts are 10 floats apart, which puts lanes u and u + 16 on one bank of a
// 32-bank dword access (2-way) and the runs of different needed ranges on further shared banks -- 7.7 conflict
// cycles per ds_read2_b32 in the sync kernel (profiles/r05/lds/lds_attrib_round4_kernel.json, tools/ubench_lds_item.hip).
// FORM 0: float2 loads (the compiler pairs them into ds_read2_b32), 1: 8-byte vector loads (paired into
// ds_read2_b64: two 16-lane accesses per half, 32 banks), 2: the same with a base VGPR per load so that they stay
// single ds_read_b64 (A/B on the reference sweep, profiles/r05/ab/mf_load_forms.txt: 0 -> 1 +0.4 %, -> 2 +0.6 %,
// conflict cycles 479 -> 351 per item).  The fixed-geometry kernel uses 2; the generic ones 1 (2 spills them at
// their 168-VGPR budget).
#ifndef FRAME_MF_B64
#define FRAME_MF_B64 3
#endif
#define FRAME_MF_B64_GEN 1
template <int ODD, int FORM, int N>
__device__ __forceinline__ void lds_readn(const float *p, int s, float (&x)[N]) {
    static_assert(N & 1, "odd window");
    if constexpr (ODD) x[0] = p[s];
    typedef const __attribute__((address_space(3))) f2v lf2c;
    lf2c *q = (lf2c *)(p + s + ODD);                     // 8-byte aligned: the caller picks ODD = parity of s
    const float2 *qf = reinterpret_cast<const float2 *>(p + s + ODD);
#pragma unroll
    for (int m = 0; m < (N - 1) / 2; ++m) {
        float wx, wy;                                    // floats s + ODD + 2m, s + ODD + 2m + 1
        if constexpr (FORM == 3) {
            const f2v w = *(volatile lf2c *)(q + m);
            wx = w.x; wy = w.y;
        } else if constexpr (FORM == 2) {
            lf2c *qm = q + m;
            opaque(qm);
            const f2v w = *qm;
            wx = w.x; wy = w.y;
        } else if constexpr (FORM == 1) {
            const f2v w = q[m];
            wx = w.x; wy = w.y;
        } else {
            const float2 w = qf[m];
            wx = w.x; wy = w.y;
        }
        x[ODD + 2 * m] = wx;
        x[ODD + 2 * m + 1] = wy;
    }
    if constexpr (!ODD) x[N - 1] = p[s + N - 1];
}


#define FRAME_CAP_U 4   // Philox blocks per lane per pass: the lazy capture's 8 + 4 blocks in passes of 4 (A/B: +1.3 % over 6, = 8)
// Capture Philox blocks bs..be (block b = waveform samples 4b..4b+3; b0 = the capture's first block) into the
// wave's region: the real parts of the clean waveform plus real AWGN (OFDM.c:622-655, D7).
// RING > 0 (frame_sync_long_kernel): the region is a ring of RING floats (a multiple of 4) plus EXT mirrored floats --
// block b goes to float 4 (b - b0) mod RING, and a block landing in [0, EXT) also to its mirror past RING, so that a
// run of <= EXT floats starting anywhere in the ring reads linearly.  Its last pass draws only ceil(rest / 64) blocks
// per lane (the matched-filter window's missing ends are 1..483 blocks long; the detection rounds' pieces fill whole
// passes either way).
template <int RING = 0, int EXT = 0, bool TRIM = false, typename A>
__device__ __forceinline__ void capture_blocks(const A &a, int wave_len, float *rbase, int b0, int bs, int be, int lane,
                                               uint32_t t_lo, uint32_t t_hi, uint32_t qs, float sigma) {
    const PhiloxHead hd = philox_head(t_lo, t_hi, STREAM_NOISE | qs, a.k1);
    const float Ksig = noise_k(sigma);
    // round keys in VGPRs: each round's two v_bitop3_b32 issue at the fast rate (an SGPR operand makes
    // them slow-class); 20 VGPRs for the capture loop only (held across the item loop instead, in
    // the fixed-geometry kernel, they spill one VGPR)
    PhiloxKeysV vk;
    vk.init(a.k0, a.k1);
    // Gaussian k of the trial's stream goes to waveform sample k (as if Transmission_Over_Air had drawn
    // the whole waveform); only the captured samples are ever evaluated.  The waveform is FR_REPS
    // copies of one filtered frame (OFDM.c:607-612): sample k is sample k mod nfilt of the first copy
    // (7.8 KB, L1-resident).  bm = the block's index within the copy.
    const uint32_t pb = (uint32_t)(wave_len / (4 * FR_REPS)), nb_wave = (uint32_t)(wave_len / 4);
    uint32_t bm = (uint32_t)(bs + lane) % pb;
    const bool real = a.noise == OFDM_NOISE_REAL;        // real-only AWGN (D7), or noiseless
    // One pass: lane l draws blocks p0 + l + 64 u, u < U, and stores those <= be.  Uniform over the wave and free of
    // per-lane control flow: every lane loads, draws and combines its U blocks (a lane past `be` computes a block it
    // does not store), so the blocks' Philox rounds and Box-Muller transcendentals interleave (ILP 2 U in the multiply
    // chains).  bm advances by 64 per block drawn.
    auto pass = [&](auto uc, int p0) {
        constexpr int U = decltype(uc)::value;
        const int bb = p0 + lane;
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int b = bb + 64 * u;
            // the block's 4 clean real parts in one 16-B load (bm < pb: inside the table; the compiler keeps it under
            // `in`, and forcing it on every lane measured 1 % slower, profiles/r04/ab/ab_ab_ntu.txt)
            const float4 re = *reinterpret_cast<const float4 *>(a.wave_re + 4 * bm);
            const bool in = (uint32_t)b < nb_wave;                     // past the waveform's end: zeros
            v[u] = in ? re : make_float4(0.f, 0.f, 0.f, 0.f);
            bm = bm + 64 >= pb ? bm + 64 - pb : bm + 64;           // (bm + 64) mod pb (pb > 64)
        }
        if (real) {         // sigma z = sqrt(K log2 u1) (cos | sin 2 pi u2) per pair
            uint32_t c2[U];
            uint4 o[U];
#pragma unroll
            for (int u = 0; u < U; ++u) c2[u] = (uint32_t)(bb + 64 * u);
            philox10_c2_multi(hd, c2, vk, o);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const Noise4 nz = noise4_of(o[u], Ksig);
                v[u].x = fmaf(nz.r0, nz.c0, v[u].x); v[u].y = fmaf(nz.r0, nz.s0, v[u].y);
                v[u].z = fmaf(nz.r1, nz.c1, v[u].z); v[u].w = fmaf(nz.r1, nz.s1, v[u].w);
            }
        }
        // samples of the block outside [0, L) land in the region's slack, never read as capture
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (bb + 64 * u <= be) {
                if constexpr (RING > 0) {
                    uint32_t pos = 4u * (uint32_t)(bb + 64 * u - b0);       // < 3 RING: two unsigned reductions
                    pos = min(pos, pos - (uint32_t)RING);
                    pos = min(pos, pos - (uint32_t)RING);
                    *reinterpret_cast<float4 *>(rbase + pos) = v[u];
                    if (pos < (uint32_t)EXT) *reinterpret_cast<float4 *>(rbase + pos + RING) = v[u];
                } else {
                    *reinterpret_cast<float4 *>(rbase + 4 * (bb + 64 * u - b0)) = v[u];
                }
            }
    };
    using U4 = std::integral_constant<int, FRAME_CAP_U>;
    if constexpr (TRIM) {
        int p0 = bs;
        for (; be - p0 >= 3 * 64; p0 += FRAME_CAP_U * 64) pass(U4{}, p0);
        if (be - p0 >= 2 * 64) pass(std::integral_constant<int, 3>{}, p0);
        else if (be - p0 >= 64) pass(std::integral_constant<int, 2>{}, p0);
        else if (be - p0 >= 0) pass(std::integral_constant<int, 1>{}, p0);
    } else {
        // whole passes, written out: the fixed kernel's max-ILP schedule is sensitive to the form (through `pass` it
        // renames its registers and issues 10 instructions more)
        for (int p0 = bs; p0 <= be; p0 += FRAME_CAP_U * 64) {
            const int bb = p0 + lane;
            float4 v[FRAME_CAP_U];
#pragma unroll
            for (int u = 0; u < FRAME_CAP_U; ++u) {
                const int b = bb + 64 * u;
                // the block's 4 clean real parts in one 16-B load (bm < pb: inside the table; the compiler keeps it under
                // `in`, and forcing it on every lane measured 1 % slower, profiles/r04/ab/ab_ab_ntu.txt)
                const float4 re = *reinterpret_cast<const float4 *>(a.wave_re + 4 * bm);
                const bool in = (uint32_t)b < nb_wave;                     // past the waveform's end: zeros
                v[u] = in ? re : make_float4(0.f, 0.f, 0.f, 0.f);
                bm = bm + 64 >= pb ? bm + 64 - pb : bm + 64;           // (bm + 64) mod pb (pb > 64)
            }
            if (real) {         // sigma z = sqrt(K log2 u1) (cos | sin 2 pi u2) per pair
                uint32_t c2[FRAME_CAP_U];
                uint4 o[FRAME_CAP_U];
#pragma unroll
                for (int u = 0; u < FRAME_CAP_U; ++u) c2[u] = (uint32_t)(bb + 64 * u);
                philox10_c2_multi(hd, c2, vk, o);
#pragma unroll
                for (int u = 0; u < FRAME_CAP_U; ++u) {
                    const Noise4 nz = noise4_of(o[u], Ksig);
                    v[u].x = fmaf(nz.r0, nz.c0, v[u].x); v[u].y = fmaf(nz.r0, nz.s0, v[u].y);
                    v[u].z = fmaf(nz.r1, nz.c1, v[u].z); v[u].w = fmaf(nz.r1, nz.s1, v[u].w);
                }
            }
            // samples of the block outside [0, L) land in the region's slack, never read as capture
#pragma unroll
            for (int u = 0; u < FRAME_CAP_U; ++u)
                if (bb + 64 * u <= be) {
                    if constexpr (RING > 0) {
                        uint32_t pos = 4u * (uint32_t)(bb + 64 * u - b0);       // < 3 RING: two unsigned reductions
                        pos = min(pos, pos - (uint32_t)RING);
                        pos = min(pos, pos - (uint32_t)RING);
                        *reinterpret_cast<float4 *>(rbase + pos) = v[u];
                        if (pos < (uint32_t)EXT) *reinterpret_cast<float4 *>(rbase + pos + RING) = v[u];
                    } else {
                        *reinterpret_cast<float4 *>(rbase + 4 * (bb + 64 * u - b0)) = v[u];
                    }
                }
        }
    }
}

#define FRAME_SYNC_MINW 3   // waves per SIMD the VGPR budget targets (LDS holds 3 blocks of 4 waves per CU)
// FIX_ND, FIX_CAP > 0: the launch geometry as compile-time constants -- n_data data symbols per frame, captures of
// FIX_CAP samples generated from the waveform (no external capture, no dumps, no word-length statistics): the
// reference message's sweep, with the detection rounds, table period, matched-filter runs and hand-off layout
// folded by the compiler.  0, 0: everything from the arguments (any message, user captures, the parity dumps).
// W: waves per block (SYNC_WAVES; 1 for long captures, whose four-wave blocks would leave one block per CU).
template <int FIX_ND, int FIX_CAP, int W = SYNC_WAVES>
__global__ __launch_bounds__(64 * W, FRAME_SYNC_MINW) void frame_sync_kernel(FrameArgs a) {
    constexpr bool FIX = FIX_ND > 0;
    constexpr int MF_FORM = FIX ? FRAME_MF_B64 : FRAME_MF_B64_GEN;   // matched-filter load form (lds_readn)
    constexpr int SYNC_WAVES = W, SYNC_THREADS = 64 * W;      // this instantiation's block
    static_assert(FIX == (FIX_CAP > 0), "both or neither");
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int L = FIX ? FIX_CAP : a.cap_len, Lc = L - 47;       // Packet_Detection length (OFDM.c:663)
    const int nfr = fr_len(FIX ? FIX_ND : a.n_data);
    const int ns = acc_slots(!FIX && a.word_stats);
    const int imt_len = FIX ? FIX_IMT_COPIES * (wave_len_for(FIX_ND) / FR_REPS) + IMT_EXT : a.imt_len;
    unsigned long long *acc = smem;                                           // [n_snr][ns]
    float *imt = reinterpret_cast<float *>(acc + a.n_snr * ns);              // imaginary parts, [imt_len]
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *rbase = imt + ((imt_len + 3) & ~3) + wv * (FIX ? wave_region_floats(FIX_CAP, FIX_ND) : a.region_floats);
    // fr[] after the capture region when !fr_in_capture (the region then ends with its 2 nfr floats)
    float2 *const fr_sep = reinterpret_cast<float2 *>(rbase + (FIX ? cap_region(FIX_CAP) : a.region_floats - 2 * nfr));
    for (int i = threadIdx.x; i < a.n_snr * ns; i += SYNC_THREADS) {
        const int k = i % ns;
        acc[i] = k == 2 ? (unsigned long long)INT64_MAX : k == 3 ? (unsigned long long)INT64_MIN : 0ull;
    }
    // the table: waveform mode imt[k] = Im wave[k mod nfilt] (every capture sample n reads imt[(rx_start + n)
    // mod nfilt]; a lane's contiguous reads start below nfilt and run at most IMT_EXT past it); an external
    // capture (ofdm_receiver, one item) its own imaginary parts, imt[n] = Im ext[n], zero past L
    for (int k = threadIdx.x; k < imt_len; k += SYNC_THREADS)
        imt[k] = !FIX && a.ext ? (k < L ? a.ext[k].y : 0.f) : a.wave[k % (FIX ? wave_len_for(FIX_ND) / FR_REPS : a.im_period)].y;
    __syncthreads();
    const int lane = threadIdx.x & 63;
#ifdef OFDM_FRAME_STAMPS
    unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long stamp_t = __builtin_amdgcn_s_memtime();
#endif
    // detection geometry (DetGeom): R rounds of 64 lanes, c0 positions per lane in round 0, c1 (+ 1 on x1 lanes)
    // in round 1 from B1
    const DetGeom dg = DetGeom::of(Lc);
    const int c0 = dg.c0, c1 = dg.c1, x1 = dg.x1, B1 = dg.B1, R = dg.R;
    auto r1_start = [c1, x1](int l) { return DetGeom::r1_start_of(c1, x1, l); };
    // Items go out in runs of FRAME_ITEM_RUN per wave: wave gw starts with run gw, the runs past the first
    // gridDim.x * SYNC_WAVES come from a per-launch atomic counter, so waves that run fast take more runs.
    // Lane 0 fetches the next run at the first item of the current one (its wait is paid once per run).
    const int nwaves = (int)gridDim.x * SYNC_WAVES;
    int64_t run_end = ((int64_t)blockIdx.x * SYNC_WAVES + wv) * FRAME_ITEM_RUN + FRAME_ITEM_RUN;
    int nxt = 0;
    int rs_run = 0;                       // lane l: the capture offset of item l of the current run
    for (int64_t i = run_end - FRAME_ITEM_RUN; i < a.n_items;) {
        // the kernel arguments are re-read per item (scalar loads through a pointer made opaque here)
        // instead of being hoisted into SGPRs held across the item loop, which spill
        using KArgs = const __attribute__((address_space(4))) FrameArgs;
        KArgs *ap = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        KArgs &a = *ap;
        // the geometry: compile-time constants (FIX), or re-read per item with the arguments
        const int n_data = FIX ? FIX_ND : a.n_data;
        const int wave_len = FIX ? wave_len_for(FIX_ND) : a.wave_len;
        const bool word_stats = !FIX && a.word_stats;
        // the imaginary-part table: period nfilt (one waveform copy) for generated captures, 2^30 for an external one
        const ImMod im_mod = FIX ? ImMod{wave_len_for(FIX_ND) / FR_REPS,
                                         (uint32_t)((((uint64_t)1 << 32) + wave_len_for(FIX_ND) / FR_REPS - 1) /
                                                    (wave_len_for(FIX_ND) / FR_REPS))}
                                 : ImMod{a.im_period, a.im_magic};
        const bool fr_in_cap = FIX ? fr_in_capture(FIX_CAP, FIX_ND) : a.fr_in_cap;
        if (lane == 0 && i == run_end - FRAME_ITEM_RUN) nxt = nwaves + (int)atomicAdd(a.work, 1ull);
        const int64_t g = a.item0 + i;
        uint32_t qr;
        const int64_t ti = a.trial0 + snr_divmod((uint32_t)a.q0 + (uint32_t)i, (uint32_t)a.n_snr, a.snr_magic, qr);
        const int q = (int)qr;
        const uint64_t t = a.first_trial + (uint64_t)ti;
        const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32), qs = (uint32_t)(a.q_base + q);
        const float sigma = a.sigma[q];
        const bool first_item = g == 0;
        const bool ext = !FIX && a.ext && first_item;
        // ---- capture window (OFDM.c:945-955) + AWGN: the real parts only ----
        int rx_start = a.fixed_start;
        if (!FIX && rx_start < 0) {        // (the generic kernel has no VGPR to spare for the run's offsets)
            const uint4 o = philox10(t_lo, t_hi, 0u, STREAM_START | qs, a.k0, a.k1);
            rx_start = (int)(o.x % (uint32_t)(wave_len - L));
        } else if (rx_start < 0) {
            // the run's FRAME_ITEM_RUN capture offsets are drawn at its first item, lane l the offset of item l of
            // the run (one Philox evaluation per run instead of one per item; the same draws)
            const int k = (int)(i - (run_end - FRAME_ITEM_RUN));
            if (k == 0) {
                uint32_t ql;
                const uint32_t tl = snr_divmod((uint32_t)a.q0 + (uint32_t)i + (uint32_t)min(lane, FRAME_ITEM_RUN - 1),
                                               (uint32_t)a.n_snr, a.snr_magic, ql);
                const uint64_t tt = a.first_trial + (uint64_t)(a.trial0 + tl);
                const uint4 o = philox10((uint32_t)tt, (uint32_t)(tt >> 32), 0u, STREAM_START | (uint32_t)(a.q_base + (int)ql),
                                         a.k0, a.k1);
                rs_run = (int)(o.x % (uint32_t)(wave_len - L));
            }
            rx_start = __builtin_amdgcn_readlane(rs_run, k);
        }
        rx_start = __builtin_amdgcn_readfirstlane(rx_start);     // uniform: the capture geometry in SGPRs
        const int off = rx_start & 3;
        const float *r = rbase + off;                       // r[n] = Re capture sample n
        // Im capture sample n = imt[im0 + n] reduced mod the period (a.im_period: nfilt, or 2^30 for ext)
        const int im0 = ext ? 0 : im_mod(rx_start);
        // lazy capture + detection (FRAME_LAZY): not for external captures, dumps or the word-length report,
        // which read the whole capture
        const bool lazy = FRAME_LAZY && !a.no_lazy && !ext && R == 2 && !word_stats &&
                          (FIX || (!a.dbg_corr && !(a.dbg_frame && first_item)));
        int b1s = 0;                                         // last Philox block generated
        if (ext) {
            for (int n = lane; n < L; n += 64) rbase[off + n] = a.ext[n].x;
        } else {
            // lazy: the blocks of capture samples [0, B1 + 47) first (round 0 reads them), the rest on demand
            const int b0 = rx_start >> 2, b1 = (rx_start + L - 1) >> 2;
            b1s = lazy ? min((rx_start + B1 + 46) >> 2, b1) : b1;
            capture_blocks(a, wave_len, rbase, b0, b0, b1s, lane, t_lo, t_hi, qs, sigma);
        }
        wave_lds_sync();
        FR_STAMP(0);                                           // capture + noise
        // lane-derived values are re-derived per item, not held across the item loop
        int lx = lane;
        opaque(lx);

        // ---- Word_Optimization_Analysis(Rx_filter_signal) (OFDM.c:38-73, 962-967): the full RRC matched
        // filter of the capture, min / max over real and imaginary parts (opt-in) ----
        if (word_stats) {
            float mn = 1e9f, mx = -1e9f;
            for (int k = lx; k < L + 20; k += 64) {
                float2 v = make_float2(0.f, 0.f);
#pragma unroll
                for (int j = 0; j < 21; ++j) {
                    const int m = k - j;
                    if (m >= 0 && m < L) {
                        const int mi = im_mod(im0 + m);
                        v.x = fmaf(r[m], a.taps[j], v.x);
                        v.y = fmaf(imt[mi], a.taps[j], v.y);
                    }
                }
                mn = fminf(mn, fminf(v.x, v.y));
                mx = fmaxf(mx, fmaxf(v.x, v.y));
            }
            mn = wave_min_f(mn);
            mx = wave_max_f(mx);
            if (lx == 0) {
                atomicMin(reinterpret_cast<long long *>(&acc[q * ns + 2]), (long long)__float2ll_rn(mn * (float)OFDM_EVM_Q_SCALE));
                atomicMax(reinterpret_cast<long long *>(&acc[q * ns + 3]), (long long)__float2ll_rn(mx * (float)OFDM_EVM_Q_SCALE));
            }
        }

        // ---- Packet_Detection (OFDM.c:659-683): M[n] = |sum r[n+k] r[n+k+16]|^2 / (sum |r[n+k+16]|^2)^2,
        // k < 32, no conjugate, on the UNFILTERED capture; sliding sums over each lane's chunk, DET_B
        // positions per batch.  M > 0.75 (OFDM.c:687, 695) is decided as the sign of
        // t = 0.75 den - num (fma: exact before its one rounding): t < 0 <=> crossing, which keeps the
        // division's outcomes 0/0 -> false (t = +0) and x/0 -> true (t = -num).  Lane l of round rho owns
        // positions [base + l chunk, +chunk) (round 0: base 0, chunk c0; round 1: B1, c1); crossing n at bit n - n0
        // of the round's mask. ----
        unsigned long long cm[2] = {0ull, 0ull};
        int first[2] = {-1, -1}, last[2] = {-1, -1};
        auto detect = [&](auto rc) {
            constexpr int rho = decltype(rc)::value;
            const int chunk = rho ? r1_start(lx + 1) - r1_start(lx) : c0;
            const int n0 = rho ? B1 + r1_start(lx) : lx * c0, n1 = min(n0 + chunk, Lc);
            unsigned long long cmask = 0ull;
            if (rho < R && n0 < n1) {
                // Im of sample n0 + k at ti_[k] (k < IMT_EXT), Re at tr_[k].  Both bases are held in one VGPR each
                // (LDS address space, made opaque), so that every block read is a ds_read2_b32 off it with an
                // immediate offset (< 1 KB) -- otherwise the compiler folds part of the table base into constants
                // too large for the offset field and spends one v_add per read on addresses
                using LdsF = const __attribute__((address_space(3))) float;
                // (the period wrap puts part of a 32-lane group on a shifted bank pattern; a timing-only build without
                // it measured no difference and 19 of 527 conflict cycles per item, profiles/r04/pmc_ab/q_lds_nowrap)
                // with FIX_IMT_COPIES >= 3 the round's base is reduced once (uniform) and the lanes read a linear run
                LdsF *ti_ = (LdsF *)(imt + (FIX && FIX_IMT_COPIES >= 3 ? (rho ? im_mod(im0 + B1) + (n0 - B1) : im0 + n0)
                                                                         : im_mod(im0 + n0)));
                LdsF *tr_ = (LdsF *)(r + n0);
                opaque(ti_);
                opaque(tr_);
                float sx = 0.f, sy = 0.f, pw = 0.f;
                uint32_t mlo = 0u, mhi = 0u;
                const int nbat = ((rho ? c1 + (x1 > 0) : c0) + DET_B - 1) / DET_B;   // uniform over the lanes
                // Samples in register blocks of DET_B: position n's window terms read samples n (leaving), n + 16,
                // n + 32 and n + 48 (entering), i.e. blocks b, b + 1, b + 2, b + 3 of batch b, so every sample is
                // loaded from LDS once (ds_read2_b32) instead of four times (A/B: +2.3 % frame mode, 167 VGPRs).
                static_assert(DET_B == 16, "blocks of 16 samples: the 16-sample lag is one block");
                constexpr int NB = 64 / DET_B;                    // batches per round at most
                float xr[NB + 3][DET_B], xi[NB + 3][DET_B];
                auto load_blk = [&](auto jc) {
                    constexpr int j = decltype(jc)::value;
#pragma unroll
                    for (int k = 0; k < DET_B; ++k) { xr[j][k] = tr_[DET_B * j + k]; xi[j][k] = ti_[DET_B * j + k]; }
                };
                load_blk(std::integral_constant<int, 0>{});
                load_blk(std::integral_constant<int, 1>{});
                load_blk(std::integral_constant<int, 2>{});
                static_for<0, 2>([&](auto hc) {                    // the first window: k = 16 h + kk
                    constexpr int h = decltype(hc)::value;
#pragma unroll
                    for (int kk = 0; kk < DET_B; ++kk) {
                        const float ux = xr[h][kk], uy = xi[h][kk], vx = xr[h + 1][kk], vy = xi[h + 1][kk];
                        sx = fmaf(ux, vx, sx); sx = fmaf(-uy, vy, sx);
                        sy = fmaf(ux, vy, sy); sy = fmaf(uy, vx, sy);
                        pw = fmaf(vx, vx, pw); pw = fmaf(vy, vy, pw);
                    }
                });
                // t's sign bits shifted in with v_alignbit, one per position (first position highest); every
                // active lane runs the same ceil(chunk / DET_B) batches, positions past n1 are masked below
                static_for<0, NB>([&](auto bc) {
                    constexpr int b = decltype(bc)::value;
                    if (b < nbat) {                                // reads past the capture stay in the region (cap_region)
                        load_blk(std::integral_constant<int, b + 3>{});
#pragma unroll
                        for (int k = 0; k < DET_B; ++k) {
                            const float o0x = xr[b][k], o0y = xi[b][k], o1x = xr[b + 1][k], o1y = xi[b + 1][k];
                            const float i0x = xr[b + 2][k], i0y = xi[b + 2][k], i1x = xr[b + 3][k], i1y = xi[b + 3][k];
                            const float num = fmaf(sx, sx, sy * sy), h = 0.75f * pw;
                            const float tt = fmaf(h, pw, -num);
                            mhi = __builtin_amdgcn_alignbit(mhi, mlo, 31);
                            mlo = __builtin_amdgcn_alignbit(mlo, __float_as_uint(tt), 31);
                            sx = fmaf(i0x, i1x, sx); sx = fmaf(-i0y, i1y, sx);
                            sx = fmaf(-o0x, o1x, sx); sx = fmaf(o0y, o1y, sx);
                            sy = fmaf(i0x, i1y, sy); sy = fmaf(i0y, i1x, sy);
                            sy = fmaf(-o0x, o1y, sy); sy = fmaf(-o0y, o1x, sy);
                            pw = fmaf(i1x, i1x, pw); pw = fmaf(i1y, i1y, pw);
                            pw = fmaf(-o1x, o1x, pw); pw = fmaf(-o1y, o1y, pw);
                        }
                    }
                });
                // J = nbat * DET_B <= 64 positions: position j sits at bit J - 1 - j of (mhi:mlo); reverse
                const int J = nbat * DET_B;
                const unsigned long long rev = ((unsigned long long)__builtin_bitreverse32(mlo) << 32) |
                                               __builtin_bitreverse32(mhi);
                cmask = rev >> (64 - J);
                cmask &= (1ull << (n1 - n0)) - 1ull;          // the last batch's positions past n1 (n1 - n0 < 64)
            }
            cm[rho] = cmask;
            first[rho] = cmask ? n0 + __builtin_ctzll(cmask) : -1;
            last[rho] = cmask ? n0 + 63 - __builtin_clzll(cmask) : -1;
        };
        // the crossing bit of position pos (< Lc) from the lane that owns it (ds_bpermute)
        auto crossing = [&](int pos) {
            const int rp = pos >= B1, rel = pos - (rp ? B1 : 0);
            int v;
            if (!rp) {
                v = rel / c0;
            } else {                                             // the lane whose round-1 chunk holds rel
                v = (rel * 64) / (64 * c1 + x1);
                if (r1_start(v + 1) <= rel) ++v;
                else if (r1_start(v) > rel) --v;
            }
            const int owner = v & 63, bit = rel - (rp ? r1_start(v) : v * c0);
            unsigned long long w = 0ull;
            static_for<0, 2>([&](auto r2c) {
                constexpr int r2 = decltype(r2c)::value;
                if (r2 < R) {
                    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)cm[r2], owner, 64);
                    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(cm[r2] >> 32), owner, 64);
                    if (rp == r2) w = ((unsigned long long)hi << 32) | lo;
                }
            });
            return ((w >> bit) & 1ull) != 0ull;
        };
        detect(std::integral_constant<int, 0>{});
        // Lazy: round 0 decides Packet_Selection when its least valid front f (M[f + 230] > 0.75 with f + 230 < B1)
        // has a later front in round 0 -- every earlier front is > 300 before f, so its own check lies in round 0
        // and failed, and neither the fronts nor their checks before f depend on round 1 -- and the matched
        // filter's samples [p - 20, p + 2 (nfr - 1) + 10] lie in the generated part.
        bool decided = false;
        int cand0 = 0x7fffffff;
        if (lazy) {
            const int pm = wave_prefix_max(last[0]);
            const int prev = max(wave_shr1(pm), -1);
            const int front = (first[0] >= 0 && first[0] - prev > 300) ? first[0] : -1;
            const int pos = front + 230;
            const bool valid = crossing(pos < B1 ? pos : 0) && front >= 0 && pos < B1;
            const int vmin0 = wave_min_i(valid ? front : 0x7fffffff), fmax0 = wave_max_i(front);
            const int gen = 4 * (b1s + 1) - rx_start;            // capture samples generated: [0, gen)
            decided = vmin0 < fmax0 && vmin0 + 11 + 2 * (nfr - 1) + 10 < gen;
            cand0 = vmin0;
        }
        if (R == 2 && !decided) {
            if (lazy) {                                          // the rest of the capture, then round 1
                capture_blocks(a, wave_len, rbase, rx_start >> 2, b1s + 1, (rx_start + L - 1) >> 2, lane, t_lo, t_hi, qs,
                               sigma);
                wave_lds_sync();
            }
            detect(std::integral_constant<int, 1>{});
        }
        if (!FIX && a.dbg_corr && first_item) {     // Corr_Out for ofdm_receiver's parity dump
            for (int n = lx; n < Lc; n += 64) {
                float sx = 0.f, sy = 0.f, pw = 0.f;
                for (int k = 0; k < 32; ++k) {
                    const float ux = r[n + k], uy = imt[im_mod(im0 + n + k)];
                    const float vx = r[n + k + 16], vy = imt[im_mod(im0 + n + k + 16)];
                    sx += ux * vx - uy * vy;
                    sy += ux * vy + uy * vx;
                    pw += vx * vx + vy * vy;
                }
                a.dbg_corr[n] = (sx * sx + sy * sy) / (pw * pw);
            }
        }
        FR_STAMP(1);                                           // packet detection

        // ---- Packet_Selection (OFDM.c:685-771): crossing idx[j] is a front iff idx[j] - idx[j-1] > 300
        // (idx[-1] = -1).  Fronts are > 300 apart and a chunk is < 300 positions, so only a lane's first
        // crossing can be one, and its predecessor is the last crossing of the earlier chunks: an exclusive
        // prefix max over (round, lane).  The first front x with a later front and M[front+230] > 0.75 gives
        // packet_idx = front + len_RRC_rx + 1; otherwise 0 (OFDM.c:752-761). ----
        int cand = cand0;
        if (!decided) {
            int vmin = 0x7fffffff, fmax_ = -1, carry = -1;
            static_for<0, 2>([&](auto rc) {
                constexpr int rho = decltype(rc)::value;
                if (rho < R) {
                    const int pm = max(wave_prefix_max(last[rho]), carry);
                    const int prev = max(wave_shr1(pm), carry);
                    const int front = (first[rho] >= 0 && first[rho] - prev > 300) ? first[rho] : -1;
                    carry = __builtin_amdgcn_readlane(pm, 63);
                    const int pos = front + 230;
                    const bool valid = crossing(pos < Lc ? pos : 0) && front >= 0 && pos < Lc;
                    vmin = min(vmin, valid ? front : 0x7fffffff);
                    fmax_ = max(fmax_, front);
                }
            });
            // the first valid front that has a later front: the least valid front, unless it is the last one
            const int cmin = wave_min_i(vmin), cmax = wave_max_i(fmax_);
            cand = cmin < cmax ? cmin : 0x7fffffff;
        }
        const bool sync_fail = cand == 0x7fffffff;
        const int p = sync_fail ? 0 : cand + 10 + 1;           // len_RRC_rx + 1 (OFDM.c:758)
        FR_STAMP(2);                                           // packet selection

        // fr[] (float2) in the unread prefix [0, off + lo) or the unread suffix (off + hi, region) of the region
        float2 *fr = fr_sep;
        if (fr_in_cap) {
            const int lo = max(p - 20, 0), hi = min(p + 2 * nfr - 2, L - 1);
            fr = off + lo >= 2 * nfr ? reinterpret_cast<float2 *>(rbase)
                                     : reinterpret_cast<float2 *>(rbase + ((off + hi + 2) & ~1));
        }
        // ---- RRC matched filter at the down-sampled instants p + 2i (OFDM.c:965, 992-996): outputs
        // interleaved over the lanes, so a tap's reads are 2 samples apart across lanes (ds_read_b64 pairs:
        // adjacent lanes read adjacent 8 B).  Only the 160 + 64 nd frame samples the receiver reads are
        // filtered (needed_k), all nfr for the single-capture dump.  The OOB flag is unchanged: the reference
        // reads past its buffer iff the last instant does, and the last sample is always needed. ----
        const bool dbg = !FIX && a.dbg_frame && first_item;
        bool oob_l = false;
        // the RRC taps are symmetric (h[t] = h[20 - t], OFDM.c:32; rrc_taps), so a window is 10 pair sums + the
        // centre tap: 11 FMAs per component instead of 21
        float tv[11];
        {
            // taps scalar-loaded from the kernarg segment per item and moved to VGPRs (an FMA with an SGPR
            // operand issues in the slow class), dying after the filter
            using kchar = __attribute__((address_space(4))) char;
            using kfloat = __attribute__((address_space(4))) float;
            const kfloat *tp = (const kfloat *)((const kchar *)__builtin_amdgcn_kernarg_segment_ptr() +
                                                offsetof(FrameArgs, taps));
            asm volatile("" : "+s"(tp));
#pragma unroll
            for (int j = 0; j < 11; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(tv[j]) : "s"(tp[j]));
        }
        // parities of the first float of a filter window in the region and in the table: uniform per item
        // (n = p + 2 ii; the period is even)
        const int par_r = (off + p) & 1, par_i = (im0 + p) & 1;
        // one output at frame instant ii (the per-instant path: windows that leave the capture, the dump)
        auto mf_one = [&](int ii) {
            const int n = p + 2 * ii;
            float2 v = make_float2(0.f, 0.f);
            if (n >= 20 && n < L) {                              // all 21 taps inside the capture
                float xr[21], xi[21];                            // x[20 - t] = sample n - t
                const int si = im_mod(im0 + n - 20);
                if (par_r) lds_readn<1, MF_FORM>(rbase, off + n - 20, xr); else lds_readn<0, MF_FORM>(rbase, off + n - 20, xr);
                if (par_i) lds_readn<1, MF_FORM>(imt, si, xi); else lds_readn<0, MF_FORM>(imt, si, xi);
                v = make_float2(xr[10] * tv[10], xi[10] * tv[10]);
#pragma unroll
                for (int tt = 0; tt < 10; ++tt) {
                    v.x = fmaf(xr[tt] + xr[20 - tt], tv[tt], v.x);
                    v.y = fmaf(xi[tt] + xi[20 - tt], tv[tt], v.y);
                }
            } else if (n >= L + 20) {
                oob_l = true;                                    // the reference reads past its buffer
            } else {
#pragma unroll
                for (int tt = 0; tt < 21; ++tt) {
                    const int m = n - tt;
                    const int mc = min(max(m, 0), L - 1);
                    const bool in = m >= 0 && m < L;
                    const float xr = in ? r[mc] : 0.f, xi = in ? imt[im_mod(im0 + mc)] : 0.f;
                    const float h = tv[tt <= 10 ? tt : 20 - tt];
                    v.x = fmaf(xr, h, v.x);
                    v.y = fmaf(xi, h, v.y);
                }
            }
            fr[ii] = v;                                          // outside every lane's reads
        };
        if (dbg) {
            for (int j = lx; j < nfr; j += 64) mf_one(j);
        } else {
            // runs of MF_RUN consecutive instants inside one needed range ([80, 112) the coarse-CFO lag window,
            // [192, 320) both LTFs, [336 + 80 d, +64) the data windows): a run's outputs share their samples, so
            // a lane loads 2 MF_RUN + 19 samples per run instead of 21 per output (58 instead of 210 LDS
            // floats for 5 outputs).  One run per lane and pass (59 runs for the reference message).
            constexpr int MF_RUN = 5, MF_W = 2 * MF_RUN + 19;
            constexpr int c0 = (32 + MF_RUN - 1) / MF_RUN, c1 = c0 + (128 + MF_RUN - 1) / MF_RUN;
            constexpr int cd = (64 + MF_RUN - 1) / MF_RUN;
            const int n_runs = c1 + cd * n_data;
            const int im_mf = im_mod(im0 + p - 20 + (wave_len / FR_REPS));      // table index of sample p - 20 (uniform)
            for (int u = lx; u < n_runs; u += 64) {
                int s0, e;
                if (u < c0) {
                    s0 = 80 + MF_RUN * u; e = 112;
                } else if (u < c1) {
                    s0 = 192 + MF_RUN * (u - c0); e = 320;
                } else {
                    const int d = (u - c1) / cd, k = u - c1 - d * cd;
                    s0 = 336 + 80 * d + MF_RUN * k; e = 400 + 80 * d;
                }
                e = min(e, s0 + MF_RUN);
                const int n_lo = p + 2 * s0 - 20;                // first sample read
                // one run: its window's real and imaginary samples (x[k] = sample n_lo + k) from float parities PR /
                // PI, then its outputs
                auto mf_run = [&](auto prc, auto pic) {
                    constexpr int PR = decltype(prc)::value, PI = decltype(pic)::value;
                    float xr[MF_W], xi[MF_W];
                    lds_readn<PR, MF_FORM>(rbase, off + n_lo, xr);
                    // with FIX_IMT_COPIES >= 3: the pass's uniform base + the lane's offset 2 s0 (< 1,000: inside the copies)
                    lds_readn<PI, MF_FORM>(imt, FIX && FIX_IMT_COPIES >= 3 ? im_mf + 2 * s0 : im_mod(im0 + n_lo), xi);
#pragma unroll
                    for (int o = 0; o < MF_RUN; ++o) {           // output at sample n_lo + 2 o + 20
                        if (s0 + o < e) {
                            float2 v = make_float2(xr[2 * o + 10] * tv[10], xi[2 * o + 10] * tv[10]);
#pragma unroll
                            for (int tt = 0; tt < 10; ++tt) {
                                v.x = fmaf(xr[2 * o + 20 - tt] + xr[2 * o + tt], tv[tt], v.x);
                                v.y = fmaf(xi[2 * o + 20 - tt] + xi[2 * o + tt], tv[tt], v.y);
                            }
                            fr[s0 + o] = v;
                        }
                    }
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                if (n_lo >= 0 && p + 2 * (e - 1) < L) {
                    if constexpr (FIX) {
                        // a generated capture: im0 = rx_start mod nfilt (even) and off = rx_start & 3 have the parity
                        // of rx_start, so par_i == par_r, and each parity is one straight-line copy of the run (no
                        // register copies where two load paths would join)
                        if (par_r) mf_run(I1{}, I1{}); else mf_run(I0{}, I0{});
                    } else {
                        if (par_r) {
                            if (par_i) mf_run(I1{}, I1{}); else mf_run(I1{}, I0{});
                        } else {
                            if (par_i) mf_run(I0{}, I1{}); else mf_run(I0{}, I0{});
                        }
                    }
                } else {
                    for (int ii = s0; ii < e; ++ii) mf_one(ii);
                }
            }
        }
        const bool oob = __ballot(oob_l) != 0ull;
        wave_lds_sync();
        FR_STAMP(3);                                           // matched filter + down-sample

        // ---- Coarse CFO (OFDM.c:773-804): 16-lag autocorrelation of the short preamble; fine CFO
        // (OFDM.c:806-828): 64-lag over the two long training symbols after the coarse rotation, the 128
        // rotated LTF samples formed on the fly (the same arithmetic as rotating the whole frame first).
        // Both estimates are wave reductions. ----
        // every fr[] sample the estimates read, loaded in one LDS round trip (lanes >= 16 read the coarse window
        // too, and drop it)
        const float2 cu = fr[80 + (lx & 15)], cw = fr[96 + (lx & 15)], l1 = fr[192 + lx], l2 = fr[256 + lx];
        float2 d0 = make_float2(0.f, 0.f), d1 = d0;          // the reference frame's data windows, for the hand-off
        if constexpr (FIX && FIX_ND == 2) {
            d0 = fr[336 + lx];
            d1 = fr[416 + lx];
        }
        float2 pp = make_float2(0.f, 0.f);
        if (lx < 16) pp = make_float2(cu.x * cw.x + cu.y * cw.y, cu.y * cw.x - cu.x * cw.y);
        pp.x = wave_sum_f(pp.x);
        pp.y = wave_sum_f(pp.y);
        double fc = (-1.0 / (2.0 * M_PI * 16.0 * TS)) * (double)atan2_cfo(pp.y, pp.x);
        if (a.float_cfo) fc = (double)(float)fc;
        {
            const float2 u = cfo_rot(l1, fc * TS, 192 + lx), w = cfo_rot(l2, fc * TS, 256 + lx);
            pp = make_float2(u.x * w.x + u.y * w.y, u.y * w.x - u.x * w.y);
        }
        pp.x = wave_sum_f(pp.x);
        pp.y = wave_sum_f(pp.y);
        double ff = (-1.0 / (2.0 * M_PI * 64.0 * TS)) * (double)atan2_cfo(pp.y, pp.x);
        if (a.float_cfo) ff = (double)(float)ff;
        // ---- coarse then fine rotation (OFDM.c:802, 825) as ONE rotation by the summed phase
        // 2 pi (fc + ff) Ts k, evaluated in fp64 revolutions (the reference's two double-precision cexp
        // products rounded to float twice; the same rotation to fp32 rounding), the result handed off
        // directly: LTF1 [192,256) + LTF2 [256,320) as one window, data d [336 + 80 d, +64) (OFDM.c:830-850,
        // 1024-1040) ----
        const int nw = 1 + n_data;
        const int ipb = FIX ? (SYM_THREADS / 4) / ((FIX_ND + 1) / 2) : a.ipb;
        float2 *dst = win_item(a.win, ipb, nw, i);
        const double fcf_ts = (fc + ff) * TS;
        // hand-off: window 0 = rot(LTF1) + rot(LTF2) sample by sample, windows 1 + d = data symbol d
        if constexpr (FIX && FIX_ND == 2) {
            // lane lx fills sample n = lx of the three windows (all four samples loaded with the CFO's): three
            // stores, each lane's 3 slots adjacent, the item's four 384-B groups whole lines once all three are done
            const float2 u = cfo_rot(l1, fcf_ts, 192 + lx), w = cfo_rot(l2, fcf_ts, 256 + lx);
            // (non-temporal stores measured neutral, profiles/r04/ab/aa_ab_nt.txt)
            float2 *o = dst + win_off(lx, ipb, nw);
            o[0] = make_float2(u.x + w.x, u.y + w.y);
            o[1] = cfo_rot(d0, fcf_ts, 336 + lx);
            o[2] = cfo_rot(d1, fcf_ts, 416 + lx);
        } else {
            if (dbg)                                           // the single-capture dump: every rotated sample
                for (int k = lx; k < nfr; k += 64) a.dbg_frame[k] = cfo_rot(fr[k], fcf_ts, k);
            // element j = sample j / nw of window j % nw (j / nw by a 16-bit reciprocal, exact for j < 64 nw <= 576)
            const uint32_t inv_nw = (65536u + (uint32_t)nw - 1u) / (uint32_t)nw;
            for (int j = lx; j < 64 * nw; j += 64) {
                const int n = (int)(((uint32_t)j * inv_nw) >> 16), w = j - n * nw;
                float2 v;
                if (w == 0) {
                    const float2 u = cfo_rot(fr[192 + n], fcf_ts, 192 + n), x = cfo_rot(fr[256 + n], fcf_ts, 256 + n);
                    v = make_float2(u.x + x.x, u.y + x.y);
                } else {
                    const int k = 336 + 80 * (w - 1) + n;
                    v = cfo_rot(fr[k], fcf_ts, k);
                }
                dst[win_off(n, ipb, nw) + w] = v;
            }
        }
        FR_STAMP(4);                                           // coarse + fine CFO + hand-off
        if (lx == 0) {
            a.info[i] = make_int4(p, sync_fail, oob, rx_start);
            if (sync_fail) atomicAdd(&acc[q * ns + 0], 1ull);
            if (oob) atomicAdd(&acc[q * ns + 1], 1ull);
            if (a.pidx_out) a.pidx_out[(int64_t)q * a.n_trials + ti] = p;
            if (!FIX && first_item && a.dbg_ints) { a.dbg_ints[0] = p; a.dbg_ints[1] = sync_fail; a.dbg_ints[2] = oob; a.dbg_ints[3] = rx_start; }
        }
        // the next item: the next one of this run, or the first of the run fetched at this run's start
        if (i + 1 < run_end) {
            ++i;
        } else {
            i = (int64_t)__builtin_amdgcn_readfirstlane(nxt) * FRAME_ITEM_RUN;
            run_end = i + FRAME_ITEM_RUN;
        }
        // the next capture overwrites this item's region: every lane is done reading it
        wave_lds_sync();
        FR_STAMP(6);                                           // hand-off
    }
#ifdef OFDM_FRAME_STAMPS
    if (lane == 0 && a.stamps)
        for (int k = 0; k < 7; ++k) atomicAdd(&a.stamps[k], stamp_acc[k]);
#endif
    __syncthreads();
    for (int k = threadIdx.x; k < a.n_snr; k += SYNC_THREADS) {
        unsigned long long *c = a.counters + k * OFDM_NCOUNTERS;
        const unsigned long long *sl = acc + k * ns;
        if (sl[0]) atomicAdd(&c[OFDM_C_SYNC_FAIL], sl[0]);
        if (sl[1]) atomicAdd(&c[OFDM_C_OOB], sl[1]);
        if (ns == 4) {          // word_stats
            atomicMin(reinterpret_cast<long long *>(&c[OFDM_C_WL_MIN_Q]), (long long)sl[2]);
            atomicMax(reinterpret_cast<long long *>(&c[OFDM_C_WL_MAX_Q]), (long long)sl[3]);
        }
    }
}

// ---------------------------------------------------------------- K4b': symbols of the synced frames
// LS estimate + CP strip + fft + ZF + slicer + demap (OFDM.c:830-1165) for a batch of items: a quad
// carries the LTF-sum window in its lane 0 (the estimate, broadcast inside the quad by DPP) and dpq data
// windows in its last dpq lanes: {LTF, LTF, D_2k, D_2k+1} for 1..2 data symbols and the reference frame's sweep,
// {LTF, D_3k, D_3k+1, D_3k+2} for 3 and 5..8 (ceil(n_data / 3) quads per item instead of ceil(n_data / 2): the
// 8-symbol message's items take 12 lanes, not 16).  The host picks dpq through the tile size a.ipb = 64 / quads per
// item (sym_quads), from which the kernel derives it back as max(2, ceil(n_data / quads)): for 4 data symbols that
// is 2 quads of {LTF, LTF, D, D}, the same 8 lanes as {LTF, D, D, D} would take.
template <bool DUMP, int FIX_ND>   // DUMP: item 0's bits / subcarriers / metrics for ofdm_receiver
#define FRAME_SYM_MINB 2   // the parity-dump instance (256 VGPRs); the sweep instances run 3 waves/SIMD (<= 168 VGPRs,
                           // no spills: round 6 A/B, profiles/r06/frame/ab_sym3.txt, frame8 +1.2 %, frame +0.5 %)
// FIX_ND > 0: n_data as a compile-time constant (the reference message's sweep: the hand-off offsets fold)
__global__ __launch_bounds__(SYM_THREADS, DUMP ? FRAME_SYM_MINB : 3) void frame_sym_kernel(FrameArgs a) {
    const int n_data = FIX_ND ? FIX_ND : a.n_data;
    __shared__ unsigned long long acc[OFDM_MAX_SNR][8];
    constexpr int DPQ_MAX = FIX_ND ? 2 : 3;
    __shared__ float part_e[SYM_THREADS / 4][DPQ_MAX];       // per quad: EVM of its data symbols
    __shared__ uint32_t part_b[SYM_THREADS / 4][DPQ_MAX], part_a[SYM_THREADS / 4][DPQ_MAX];
    for (int k = threadIdx.x; k < a.n_snr * 8; k += SYM_THREADS) (&acc[0][0])[k] = 0ull;
    __syncthreads();
    const int lane = threadIdx.x & 63, quad = threadIdx.x >> 2, role = lane & 3;
    // quads per item and data lanes per quad: 2 with FIX_ND, else from the tile size (sym_quads)
    const int qpi = FIX_ND ? (FIX_ND + 1) / 2 : (SYM_THREADS / 4) / a.ipb;
    const int dpq = FIX_ND ? 2 : max(2, (n_data + qpi - 1) / qpi), r0 = 4 - dpq;   // first data role
    // items never straddle a wave: a wave's 16 quads carry 16 / qpi whole items (qpi = 3: 5 items, one idle quad)
    const int ipw = 16 / qpi, ipb = 4 * ipw;                               // items per wave, per block
    const int wq = quad & 15, item_l = (quad >> 4) * ipw + wq / qpi, qi = wq - (wq / qpi) * qpi;
    const int dsym = dpq == 2 ? 2 * qi + (role & 1) : 3 * qi + max(role - 1, 0);
    const int nw = 1 + n_data;
    const int dsc = min(dsym, n_data - 1);
    // role 0: the LTF-sum window (with dpq = 2 role 1 reads the same addresses and its transform is not used);
    // roles r0..3: data
    const int w = role < r0 ? 0 : 1 + dsc;
    for (int64_t base = (int64_t)blockIdx.x * ipb; base < a.n_items; base += (int64_t)gridDim.x * ipb) {
        const int64_t i = base + item_l;
        const bool item_ok = wq < ipw * qpi && i < a.n_items;
        const bool dlane = item_ok && role >= r0 && dsym < n_data;
        const float2 *src = win_item(a.win, ipb, nw, item_ok ? i : base) + w;
        float2 x[64];
#define FRAME_SYM_GROUPS 2      // hand-off groups loaded per batch of first radix-4 stages (A/B: 2 +0.4 % over 1; 4
                                // needs 172 VGPRs, 2 waves/SIMD, and gains nothing; profiles/r04/ab/x_ab_groups.txt)
        // load fused with the first radix-4 stage, FRAME_SYM_GROUPS x 16 samples (hand-off groups) at a time
        // (fft() = DFT(x (-1)^n))
        static_for<0, 4>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            gcf2 *sp = (gcf2 *)src;
            opaque(sp);
            static_for<0, 16>([&](auto pc) {
                constexpr int n = 16 * (decltype(pc)::value >> 2) + 4 * g + (decltype(pc)::value & 3);
                const float2 v = gld(sp, win_off(n, ipb, nw));
                x[n] = (n & 1) ? make_float2(-v.x, -v.y) : v;
            });
            if constexpr ((g + 1) % FRAME_SYM_GROUPS == 0) {
                static_for<0, 4 * FRAME_SYM_GROUPS>([&](auto ic) {
                    dif_stage1<false, 4 * (g + 1 - FRAME_SYM_GROUPS) + decltype(ic)::value>(x);
                });
                sched_fence();
            }
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
        if (role >= r0) {
            const int sl = dpq == 2 ? role & 1 : role - 1;
            part_e[quad][sl] = dlane ? finish_evm<2>(st) : 0.f;
            part_b[quad][sl] = dlane ? st.be : 0u;
            part_a[quad][sl] = dlane ? st.ax : 0u;
        }
        if (DUMP && dump && a.dbg_bits) { a.dbg_bits[3 * dsym] = st.d[0]; a.dbg_bits[3 * dsym + 1] = st.d[1]; a.dbg_bits[3 * dsym + 2] = st.d[2]; }
        // an item's quads are in one wave (ipw whole items per wave), so its totals need a wave's sync, not the block's
        // (round 6 A/Bs: profiles/r06/frame/ab_symws.txt, frame +0.5 %; ab_sym3.txt, with whole items per wave for
        // 3-quad items, frame8 +0.5 % over 3 waves/SIMD alone; an L2 warm-up of the block's next tile, ab_sym.txt: -3 %)
        if constexpr (!DUMP) wave_lds_sync(); else __syncthreads();
        if (item_ok && qi == 0 && role == 0) {
            // the item's totals in symbol order (deterministic), then the trial's metrics
            float fe = 0.f;
            uint32_t ferr = 0u, fax = 0u;
            for (int k = 0; k < qpi; ++k)
                for (int r2 = 0; r2 < dpq; ++r2) {
                    fe += part_e[quad + k][r2]; ferr += part_b[quad + k][r2]; fax += part_a[quad + k][r2];
                }
            const int64_t g = a.item0 + i;
            uint32_t q;
            (void)snr_divmod((uint32_t)a.q0 + (uint32_t)i, (uint32_t)a.n_snr, a.snr_magic, q);
            unsigned long long *sl = acc[q];
            atomicAdd(&sl[0], (unsigned long long)ferr);
            atomicAdd(&sl[1], (unsigned long long)(ferr > 0u));
            atomicAdd(&sl[2], (unsigned long long)fax);
            const float N = 48.0f * (float)n_data;
            atomicAdd(&sl[5], (unsigned long long)(int64_t)__float2ll_rn(fe * (float)OFDM_EVM_Q_SCALE));
            const float db = fe > 0.f ? fmaxf(3.01029995663981195214f * __builtin_amdgcn_logf(fe / N), -400.f) : -400.f;
            atomicAdd(&sl[6], (unsigned long long)(int64_t)__float2ll_rn(db * (float)OFDM_EVM_Q_SCALE));
            float dbp = -INFINITY;
            if (fax > 0u) {
                dbp = 3.01029995663981195214f * __builtin_amdgcn_logf(2.0f * (float)fax / N);
                atomicAdd(&sl[7], (unsigned long long)(int64_t)__float2ll_rn(dbp * (float)OFDM_EVM_Q_SCALE));
                atomicAdd(&sl[4], 1ull);
            }
            if (DUMP && g == 0 && a.dbg_res) { a.dbg_res[0] = db; a.dbg_res[1] = dbp; a.dbg_res[2] = (float)ferr / (96.0f * n_data); }
        }
        if constexpr (!DUMP) wave_lds_sync(); else __syncthreads();
    }
    if constexpr (!DUMP) __syncthreads();     // every wave's counter adds are in before the flush
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

static unsigned occupancy_grid(const void *kernel, int threads, size_t lds, int cus, int64_t blocks, int waves = 2) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 2;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)per_cu * cus * waves));
}

#ifdef OFDM_FRAME_SYM_TU
// K4b' (frame_sym_kernel) is instantiated in its own translation unit (ofdm_frame_sym.hip) so that the sync
// kernel's can be compiled with another scheduler (build_lib.SOURCE_FLAGS); this is its launcher.
void launch_frame_sym(hipStream_t st, const FrameArgs &a, int cus) {
    const int ipb = a.ipb;
    const bool dump = a.dbg_eq || a.dbg_bits || a.dbg_res;
    const bool sym2 = a.n_data == 2 && !getenv("OFDM_FRAME_GENERIC");     // the hand-off offsets folded
    const void *k = dump ? reinterpret_cast<const void *>(&frame_sym_kernel<true, 0>)
                  : sym2 ? reinterpret_cast<const void *>(&frame_sym_kernel<false, 2>)
                         : reinterpret_cast<const void *>(&frame_sym_kernel<false, 0>);
    const dim3 grid(occupancy_grid(k, SYM_THREADS, 0, cus, (a.n_items + ipb - 1) / ipb));
    if (dump) hipLaunchKernelGGL((frame_sym_kernel<true, 0>), grid, dim3(SYM_THREADS), 0, st, a);
    else if (sym2) hipLaunchKernelGGL((frame_sym_kernel<false, 2>), grid, dim3(SYM_THREADS), 0, st, a);
    else hipLaunchKernelGGL((frame_sym_kernel<false, 0>), grid, dim3(SYM_THREADS), 0, st, a);
}
}  // namespace ofdm
#elif defined(OFDM_FRAME_FIX_TU)
// K4b with the reference message's geometry folded (frame_sync_kernel<2, 3008>) in its own translation unit
// (ofdm_frame_fix.hip), scheduled for ILP without spilling the generic instantiations (A/B +0.4 %,
// profiles/r04/ab/q_ab_syncilp.txt); its occupancy handle and launcher
const void *frame_fix_kernel() { return reinterpret_cast<const void *>(&frame_sync_kernel<2, 3008, FIX_W>); }
void launch_frame_fix(hipStream_t st, const FrameArgs &a, dim3 grid, size_t lds) {
    hipLaunchKernelGGL((frame_sync_kernel<2, 3008, FIX_W>), grid, dim3(64 * FIX_W), lds, st, a);
}
}  // namespace ofdm
#elif defined(OFDM_FRAME_LONG_TU)
// ---------------------------------------------------------------- K4b for long captures
// Frames of 5..8 data symbols (ofdm_set_message) give captures of 4,482..5,955 samples: 18-24 KB of real parts per
// wave, so frame_sync_kernel<0, 0> fits one four-wave block per CU (1 wave per SIMD).  This kernel keeps the capture
// in a ring of LW_RING = 2,976 floats per wave (+ a 96-float mirror: 12 KB, twelve waves per CU, 3 per SIMD) that
// always holds the last 2,973 samples generated, detects in rounds of 64 lanes x 31 positions (LW_ROUND = 1,984
// positions, LW_PIECE = 2,031 samples each) and generates the capture a round at a time, all from the same
// counter-based Philox stream as the whole capture:
//   1. round 0's samples [0, 2,031) -> round 0; round 1's [1,984, 4,015) -> round 1 (two frame periods);
//   2. lazy (as frame_sync_kernel's, one round later): Packet_Selection is decided by rounds 0 and 1 when their
//      least valid front (its +230 check inside them) has a later front inside them: fronts and checks depend
//      only on earlier positions, and every later front lies past it.  Then round 2 and its samples are skipped;
//      the rounds' crossing masks stay in registers, so the rule needs no samples;
//   3. otherwise round 2's samples [3,968, L) -> round 2 and the selection over all three rounds (a.no_lazy: always);
//   4. the samples the matched filter's runs read, [p + 140, p + 2 (nfr - 1) + 10] (1,789 for 8 data symbols): the
//      part the ring does not hold is generated (57 % of the bench's items; 2.41 Philox blocks per lane and item on
//      average, the last pass trimmed to the blocks it stores; profiles/r06/frame/ab_regen.txt).
// Reads index the ring ((n + off) mod LW_RING): a lane's detection run (80 floats) and a matched-filter run (29) read
// linearly through the mirror.  Round 6 A/Bs (profiles/r06/frame/ab_long12.txt, ab_ring.txt): two rounds resident
// (16 KB per wave) in 9-wave blocks, 3, 2, 2, 2 waves on a CU's SIMDs 8.34-8.38e8; one round's piece in 12-wave blocks,
// the whole window generated again 8.58-8.62e8; the ring 8.76-8.78e8.
// The filtered frame fr[] then overwrites the region: a lane holds its runs' outputs in registers until every
// lane's reads are done.  Packet detection / selection, the matched filter, CFO and hand-off are the generic
// kernel's arithmetic, so every counter and packet_idx equals frame_sync_kernel<0, 0>'s
// (tests/test_gpu_frame.py::test_long_capture_kernel_equals_generic).  Sweeps only (generated captures, no
// dumps, no word-length statistics); no lazy capture (for long frames round 0 never decides: two fronts are one
// frame period, >= 1,940 positions, apart).
constexpr int LW_CHUNK = 31;
constexpr int LW_ROUND = 64 * LW_CHUNK;              // 1,984 positions per round
constexpr int LW_PIECE = LW_ROUND + 47;               // a round's samples: its positions and their 47-sample windows
constexpr int LW_RING = 2976, LW_EXT = 96;             // the capture ring (floats, a multiple of 4) and its mirror
constexpr int LW_MAXP = 3;                            // matched-filter passes of 64 runs (33 + 13 nd <= 137 runs)
#define FRAME_MF_B64_LONG FRAME_MF_B64_GEN   // lds_readn form of the long kernel's matched filter
template <int W>
__global__ __launch_bounds__(64 * W, FRAME_LONG_MINW) void frame_sync_long_kernel(FrameArgs a) {
    constexpr int SYNC_WAVES_L = W, SYNC_THREADS_L = 64 * W;
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int L = a.cap_len, Lc = L - 47;
    const int nfr = fr_len(a.n_data);
    constexpr int ns = 2;
    unsigned long long *acc = smem;                                           // [n_snr][2]
    float *imt = reinterpret_cast<float *>(acc + a.n_snr * ns);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *rbase = imt + ((a.imt_len + 3) & ~3) + wv * a.region_floats;
    for (int i = threadIdx.x; i < a.n_snr * ns; i += SYNC_THREADS_L) acc[i] = 0ull;
    // the imaginary parts over one period + LONG_TABLE_REACH (a.imt_len, set by the host): each detection round and
    // the matched filter reduce one uniform table base, no lane reads across the period wrap (frame_sync_kernel's
    // FIX_IMT_COPIES)
    for (int k = threadIdx.x; k < a.imt_len; k += SYNC_THREADS_L) imt[k] = a.wave[k % a.im_period].y;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int R = (Lc + LW_ROUND - 1) / LW_ROUND;                            // 2 or 3 rounds (host-checked)
    const int nwaves = (int)gridDim.x * SYNC_WAVES_L;
    int64_t run_end = ((int64_t)blockIdx.x * SYNC_WAVES_L + wv) * FRAME_ITEM_RUN + FRAME_ITEM_RUN;
    int nxt = 0;
    for (int64_t i = run_end - FRAME_ITEM_RUN; i < a.n_items;) {
        using KArgs = const __attribute__((address_space(4))) FrameArgs;
        KArgs *ap = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        KArgs &a = *ap;
        const int n_data = a.n_data, wave_len = a.wave_len;
        const ImMod im_mod{a.im_period, a.im_magic};
        if (lane == 0 && i == run_end - FRAME_ITEM_RUN) nxt = nwaves + (int)atomicAdd(a.work, 1ull);
        uint32_t qr;
        const int64_t ti = a.trial0 + snr_divmod((uint32_t)a.q0 + (uint32_t)i, (uint32_t)a.n_snr, a.snr_magic, qr);
        const int q = (int)qr;
        const uint64_t t = a.first_trial + (uint64_t)ti;
        const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32), qs = (uint32_t)(a.q_base + q);
        const float sigma = a.sigma[q];
        int rx_start = a.fixed_start;
        if (rx_start < 0) {
            const uint4 o = philox10(t_lo, t_hi, 0u, STREAM_START | qs, a.k0, a.k1);
            rx_start = (int)(o.x % (uint32_t)(wave_len - L));
        }
        rx_start = __builtin_amdgcn_readfirstlane(rx_start);
        const int off = rx_start & 3, b0 = rx_start >> 2;
        // capture sample n lives at ring float (n + off) mod LW_RING (and its mirror past LW_RING when < LW_EXT)
        auto ring = [&](int n) {
            uint32_t x = (uint32_t)(n + off);
            x = min(x, x - (uint32_t)LW_RING);
            return (int)min(x, x - (uint32_t)LW_RING);
        };
        // samples [n_lo, n_hi) into the ring (whole Philox blocks: up to 3 samples either side, with their own values)
        auto gen = [&](int n_lo, int n_hi, auto trim) {
            capture_blocks<LW_RING, LW_EXT, decltype(trim)::value>(a, wave_len, rbase, b0, (rx_start + n_lo) >> 2,
                                                                  (rx_start + n_hi - 1) >> 2, lane, t_lo, t_hi, qs, sigma);
        };
        const int im0 = im_mod(rx_start);
        int lx = lane;
        opaque(lx);
        // ---- Packet_Detection (OFDM.c:659-683) in rounds of LW_ROUND positions, lane l of round rho owning
        // [rho LW_ROUND + 31 l, +31) -- frame_sync_kernel's sliding sums and sign-bit crossings; rp: this round's
        // view of the capture (sample n at rp[n]) ----
        unsigned long long cm[3] = {0ull, 0ull, 0ull};
        int first[3] = {-1, -1, -1}, last[3] = {-1, -1, -1};
        auto detect = [&](auto rc) {
            constexpr int rho = decltype(rc)::value;
            const int n0 = rho * LW_ROUND + lx * LW_CHUNK, n1 = min(n0 + LW_CHUNK, Lc);
            unsigned long long cmask = 0ull;
            if (n0 < n1) {
                using LdsF = const __attribute__((address_space(3))) float;
                LdsF *ti_ = (LdsF *)(imt + im_mod(im0 + rho * LW_ROUND) + lx * LW_CHUNK);   // uniform base + lane offset
                LdsF *tr_ = (LdsF *)(rbase + ring(n0));                 // 80 floats: inside ring + mirror
                opaque(ti_);
                opaque(tr_);
                float sx = 0.f, sy = 0.f, pw = 0.f;
                uint32_t mlo = 0u, mhi = 0u;
                constexpr int nbat = (LW_CHUNK + DET_B - 1) / DET_B;
                float xr[nbat + 3][DET_B], xi[nbat + 3][DET_B];
                auto load_blk = [&](auto jc) {
                    constexpr int j = decltype(jc)::value;
#pragma unroll
                    for (int k = 0; k < DET_B; ++k) { xr[j][k] = tr_[DET_B * j + k]; xi[j][k] = ti_[DET_B * j + k]; }
                };
                load_blk(std::integral_constant<int, 0>{});
                load_blk(std::integral_constant<int, 1>{});
                load_blk(std::integral_constant<int, 2>{});
                static_for<0, 2>([&](auto hc) {
                    constexpr int h = decltype(hc)::value;
#pragma unroll
                    for (int kk = 0; kk < DET_B; ++kk) {
                        const float ux = xr[h][kk], uy = xi[h][kk], vx = xr[h + 1][kk], vy = xi[h + 1][kk];
                        sx = fmaf(ux, vx, sx); sx = fmaf(-uy, vy, sx);
                        sy = fmaf(ux, vy, sy); sy = fmaf(uy, vx, sy);
                        pw = fmaf(vx, vx, pw); pw = fmaf(vy, vy, pw);
                    }
                });
                static_for<0, nbat>([&](auto bc) {
                    constexpr int b = decltype(bc)::value;
                    load_blk(std::integral_constant<int, b + 3>{});
#pragma unroll
                    for (int k = 0; k < DET_B; ++k) {
                        const float o0x = xr[b][k], o0y = xi[b][k], o1x = xr[b + 1][k], o1y = xi[b + 1][k];
                        const float i0x = xr[b + 2][k], i0y = xi[b + 2][k], i1x = xr[b + 3][k], i1y = xi[b + 3][k];
                        const float num = fmaf(sx, sx, sy * sy), h = 0.75f * pw;
                        const float tt = fmaf(h, pw, -num);
                        mhi = __builtin_amdgcn_alignbit(mhi, mlo, 31);
                        mlo = __builtin_amdgcn_alignbit(mlo, __float_as_uint(tt), 31);
                        sx = fmaf(i0x, i1x, sx); sx = fmaf(-i0y, i1y, sx);
                        sx = fmaf(-o0x, o1x, sx); sx = fmaf(o0y, o1y, sx);
                        sy = fmaf(i0x, i1y, sy); sy = fmaf(i0y, i1x, sy);
                        sy = fmaf(-o0x, o1y, sy); sy = fmaf(-o0y, o1x, sy);
                        pw = fmaf(i1x, i1x, pw); pw = fmaf(i1y, i1y, pw);
                        pw = fmaf(-o1x, o1x, pw); pw = fmaf(-o1y, o1y, pw);
                    }
                });
                constexpr int J = nbat * DET_B;
                const unsigned long long rev = ((unsigned long long)__builtin_bitreverse32(mlo) << 32) |
                                               __builtin_bitreverse32(mhi);
                cmask = rev >> (64 - J);
                cmask &= (1ull << (n1 - n0)) - 1ull;
            }
            cm[rho] = cmask;
            first[rho] = cmask ? n0 + __builtin_ctzll(cmask) : -1;
            last[rho] = cmask ? n0 + 63 - __builtin_clzll(cmask) : -1;
        };
        // round rho's piece: samples [rho LW_ROUND, min(L, rho LW_ROUND + LW_PIECE)), the ring then holding the last
        // LW_RING - 3 samples generated
        auto piece = [&](int rho) { gen(rho * LW_ROUND, min(L, rho * LW_ROUND + LW_PIECE), std::false_type{}); };
        piece(0);
        wave_lds_sync();
        detect(std::integral_constant<int, 0>{});
        wave_lds_sync();                                      // round 0's loads are done: round 1's piece overwrites
        piece(1);
        wave_lds_sync();
        detect(std::integral_constant<int, 1>{});
        // the crossing bit of position pos (< Lc) from the lane that owns it (ds_bpermute)
        auto crossing = [&](int pos) {
            const int rd = pos / LW_ROUND, rel = pos - rd * LW_ROUND;
            const int owner = rel / LW_CHUNK, bit = rel - owner * LW_CHUNK;
            unsigned long long w = 0ull;
            static_for<0, 3>([&](auto r2c) {
                constexpr int r2 = decltype(r2c)::value;
                if (r2 < R) {
                    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)cm[r2], owner, 64);
                    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(cm[r2] >> 32), owner, 64);
                    if (rd == r2) w = ((unsigned long long)hi << 32) | lo;
                }
            });
            return ((w >> bit) & 1ull) != 0ull;
        };
        // ---- Packet_Selection (OFDM.c:685-771) over the first nr rounds (frame_sync_kernel's rule); a front whose
        // +230 check lies at or past `limit` is not valid (not known yet) ----
        auto select = [&](int nr, int limit) {
            int vmin = 0x7fffffff, fmax_ = -1, carry = -1;
            static_for<0, 3>([&](auto rc) {
                constexpr int rho = decltype(rc)::value;
                if (rho < nr) {
                    const int pm = max(wave_prefix_max(last[rho]), carry);
                    const int prev = max(wave_shr1(pm), carry);
                    const int front = (first[rho] >= 0 && first[rho] - prev > 300) ? first[rho] : -1;
                    carry = __builtin_amdgcn_readlane(pm, 63);
                    const int pos = front + 230;
                    const bool valid = crossing(pos < limit ? pos : 0) && front >= 0 && pos < limit;
                    vmin = min(vmin, valid ? front : 0x7fffffff);
                    fmax_ = max(fmax_, front);
                }
            });
            const int cmin = wave_min_i(vmin), cmax = wave_max_i(fmax_);
            return cmin < cmax ? cmin : 0x7fffffff;
        };
        // lazy: rounds 0 and 1 decide when their least valid front has a later front in them (the full rule then
        // picks the same front: see the header); otherwise round 2 over the region and the selection over all rounds
        int cand = R == 3 && !a.no_lazy ? select(2, min(2 * LW_ROUND, Lc)) : 0x7fffffff;
        int held = 1;                                         // the round whose piece the region holds
        if (cand == 0x7fffffff) {
            if (R == 3) {
                wave_lds_sync();                              // round 1's loads are done: round 2's piece overwrites
                piece(2);
                wave_lds_sync();
                detect(std::integral_constant<int, 2>{});
                held = 2;
            }
            cand = select(R, Lc);
        }
        const bool sync_fail = cand == 0x7fffffff;
        const int p = sync_fail ? 0 : cand + 10 + 1;
        // ---- the matched filter's samples [p + 140, p + 2 (nfr - 1) + 10] (at most 1,789 < LW_RING - 6; the first
        // instant read is frame sample 80, the STF's last 32 samples, whose window starts at p + 2 x 80 - 20): the ring
        // holds [res_lo, res_hi) of them after the last round's piece; the missing end of the window is generated --
        // forward past res_hi (evicting only samples before the window) or backward below res_lo (evicting only samples
        // past it), its last capture pass only as many blocks per lane as it stores.  A failed sync (p = 0) reads
        // [140, 2 nfr + 8]. ----
        constexpr int MF_S_FIRST = 80;                        // the first run's first instant (the runs below)
        {
            const int lo = p + 2 * MF_S_FIRST - 20, hi = min(p + 2 * (nfr - 1) + 10, L - 1);
            const int res_hi = min(L, held * LW_ROUND + LW_PIECE), res_lo = res_hi + 3 - LW_RING;
            if (hi >= res_hi || lo < res_lo) {
                wave_lds_sync();                              // detection's loads are done
                const bool fwd = hi >= res_hi;
                gen(fwd ? max(lo, res_hi) : lo, fwd ? hi + 1 : min(hi + 1, res_lo), std::true_type{});
                wave_lds_sync();
            }
        }
        // ---- RRC matched filter at the needed instants (frame_sync_kernel's runs), outputs held in registers ----
        bool oob_l = false;
        float tv[11];
        {
            using kchar = __attribute__((address_space(4))) char;
            using kfloat = __attribute__((address_space(4))) float;
            const kfloat *tp = (const kfloat *)((const kchar *)__builtin_amdgcn_kernarg_segment_ptr() +
                                                offsetof(FrameArgs, taps));
            asm volatile("" : "+s"(tp));
#pragma unroll
            for (int j = 0; j < 11; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(tv[j]) : "s"(tp[j]));
        }
        const int par_r = (off + p) & 1, par_i = (im0 + p) & 1;    // ring floats keep the parity (LW_RING even)
        constexpr int MF_RUN = 5, MF_W = 2 * MF_RUN + 19;
        constexpr int c0r = (32 + MF_RUN - 1) / MF_RUN, c1r = c0r + (128 + MF_RUN - 1) / MF_RUN;
        constexpr int cd = (64 + MF_RUN - 1) / MF_RUN;
        const int n_runs = c1r + cd * n_data;
        const int im_mf = im_mod(im0 + p - 20 + a.im_period);    // table index of sample p - 20 (uniform)
        float2 mfo[LW_MAXP][MF_RUN];
        int mfs[LW_MAXP], mfe[LW_MAXP];
        static_for<0, LW_MAXP>([&](auto pc) {
            constexpr int pi = decltype(pc)::value;
            const int u = lx + 64 * pi;
            int s0 = 0, e = 0;
            if (u < n_runs) {
                if (u < c0r) {
                    s0 = MF_S_FIRST + MF_RUN * u; e = 112;
                } else if (u < c1r) {
                    s0 = 192 + MF_RUN * (u - c0r); e = 320;
                } else {
                    const int d = (u - c1r) / cd, k = u - c1r - d * cd;
                    s0 = 336 + 80 * d + MF_RUN * k; e = 400 + 80 * d;
                }
                e = min(e, s0 + MF_RUN);
            }
            mfs[pi] = s0;
            mfe[pi] = e;
            const int n_lo = p + 2 * s0 - 20;
            if (u < n_runs && n_lo >= 0 && p + 2 * (e - 1) < L) {
                float xr[MF_W], xi[MF_W];
                const int si = im_mf + 2 * s0;                                // < 3 periods: inside the copies
                const int rl = ring(n_lo);                                    // 29 floats: inside ring + mirror
                if (par_r) lds_readn<1, FRAME_MF_B64_LONG>(rbase, rl, xr); else lds_readn<0, FRAME_MF_B64_LONG>(rbase, rl, xr);
                if (par_i) lds_readn<1, FRAME_MF_B64_LONG>(imt, si, xi); else lds_readn<0, FRAME_MF_B64_LONG>(imt, si, xi);
#pragma unroll
                for (int o = 0; o < MF_RUN; ++o) {
                    float2 v = make_float2(xr[2 * o + 10] * tv[10], xi[2 * o + 10] * tv[10]);
#pragma unroll
                    for (int tt = 0; tt < 10; ++tt) {
                        v.x = fmaf(xr[2 * o + 20 - tt] + xr[2 * o + tt], tv[tt], v.x);
                        v.y = fmaf(xi[2 * o + 20 - tt] + xi[2 * o + tt], tv[tt], v.y);
                    }
                    mfo[pi][o] = v;
                }
            } else {
#pragma unroll
                for (int o = 0; o < MF_RUN; ++o) {           // the per-instant path (windows leaving the capture)
                    const int n = p + 2 * (s0 + o);
                    float2 v = make_float2(0.f, 0.f);
                    if (u < n_runs && s0 + o < e) {
                        if (n >= L + 20) {
                            oob_l = true;
                        } else {
                            for (int tt = 0; tt < 21; ++tt) {
                                const int m = n - tt;
                                const int mc = min(max(m, 0), L - 1);
                                const bool in = m >= 0 && m < L;
                                const float xr = in ? rbase[ring(mc)] : 0.f, xi = in ? imt[im_mod(im0 + mc)] : 0.f;
                                const float h = tv[tt <= 10 ? tt : 20 - tt];
                                v.x = fmaf(xr, h, v.x);
                                v.y = fmaf(xi, h, v.y);
                            }
                        }
                    }
                    mfo[pi][o] = v;
                }
            }
        });
        const bool oob = __ballot(oob_l) != 0ull;
        wave_lds_sync();                                      // every lane's capture reads are done
        float2 *fr = reinterpret_cast<float2 *>(rbase);       // fr[] overwrites the region
        static_for<0, LW_MAXP>([&](auto pc) {
            constexpr int pi = decltype(pc)::value;
#pragma unroll
            for (int o = 0; o < MF_RUN; ++o)
                if (mfs[pi] + o < mfe[pi]) fr[mfs[pi] + o] = mfo[pi][o];
        });
        wave_lds_sync();
        // ---- coarse / fine CFO and the hand-off (frame_sync_kernel's generic path) ----
        const float2 cu = fr[80 + (lx & 15)], cw = fr[96 + (lx & 15)], l1 = fr[192 + lx], l2 = fr[256 + lx];
        float2 pp = make_float2(0.f, 0.f);
        if (lx < 16) pp = make_float2(cu.x * cw.x + cu.y * cw.y, cu.y * cw.x - cu.x * cw.y);
        pp.x = wave_sum_f(pp.x);
        pp.y = wave_sum_f(pp.y);
        double fc = (-1.0 / (2.0 * M_PI * 16.0 * TS)) * (double)atan2_cfo(pp.y, pp.x);
        if (a.float_cfo) fc = (double)(float)fc;
        {
            const float2 u = cfo_rot(l1, fc * TS, 192 + lx), w = cfo_rot(l2, fc * TS, 256 + lx);
            pp = make_float2(u.x * w.x + u.y * w.y, u.y * w.x - u.x * w.y);
        }
        pp.x = wave_sum_f(pp.x);
        pp.y = wave_sum_f(pp.y);
        double ff = (-1.0 / (2.0 * M_PI * 64.0 * TS)) * (double)atan2_cfo(pp.y, pp.x);
        if (a.float_cfo) ff = (double)(float)ff;
        const int nw = 1 + n_data;
        float2 *dst = win_item(a.win, a.ipb, nw, i);
        const double fcf_ts = (fc + ff) * TS;
        const uint32_t inv_nw = (65536u + (uint32_t)nw - 1u) / (uint32_t)nw;
        for (int j = lx; j < 64 * nw; j += 64) {
            const int n = (int)(((uint32_t)j * inv_nw) >> 16), w = j - n * nw;
            float2 v;
            if (w == 0) {
                const float2 u = cfo_rot(fr[192 + n], fcf_ts, 192 + n), x = cfo_rot(fr[256 + n], fcf_ts, 256 + n);
                v = make_float2(u.x + x.x, u.y + x.y);
            } else {
                const int k = 336 + 80 * (w - 1) + n;
                v = cfo_rot(fr[k], fcf_ts, k);
            }
            dst[win_off(n, a.ipb, nw) + w] = v;
        }
        if (lx == 0) {
            a.info[i] = make_int4(p, sync_fail, oob, rx_start);
            if (sync_fail) atomicAdd(&acc[q * ns + 0], 1ull);
            if (oob) atomicAdd(&acc[q * ns + 1], 1ull);
            if (a.pidx_out) a.pidx_out[(int64_t)q * a.n_trials + ti] = p;
        }
        if (i + 1 < run_end) {
            ++i;
        } else {
            i = (int64_t)__builtin_amdgcn_readfirstlane(nxt) * FRAME_ITEM_RUN;
            run_end = i + FRAME_ITEM_RUN;
        }
        wave_lds_sync();                                      // the next capture overwrites this item's region
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.n_snr; k += SYNC_THREADS_L) {
        unsigned long long *c = a.counters + k * OFDM_NCOUNTERS;
        const unsigned long long *sl = acc + k * ns;
        if (sl[0]) atomicAdd(&c[OFDM_C_SYNC_FAIL], sl[0]);
        if (sl[1]) atomicAdd(&c[OFDM_C_OOB], sl[1]);
    }
}

// launcher and occupancy handle (ofdm_frame_long.hip)
const void *frame_long_kernel() { return reinterpret_cast<const void *>(&frame_sync_long_kernel<LONG_W>); }
void launch_frame_long(hipStream_t st, const FrameArgs &a, dim3 grid, size_t lds) {
    hipLaunchKernelGGL((frame_sync_long_kernel<LONG_W>), grid, dim3(64 * LONG_W), lds, st, a);
}
}  // namespace ofdm
#else
void launch_frame_sym(hipStream_t st, const FrameArgs &a, int cus);     // ofdm_frame_sym.hip
const void *frame_fix_kernel();                                         // ofdm_frame_fix.hip
void launch_frame_fix(hipStream_t st, const FrameArgs &a, dim3 grid, size_t lds);
const void *frame_long_kernel();                                        // ofdm_frame_long.hip
void launch_frame_long(hipStream_t st, const FrameArgs &a, dim3 grid, size_t lds);
// the long-capture kernel's per-wave region (floats): the capture ring and its mirror, then fr[]
constexpr int FRAME_LONG_REGION = 3072;                // LW_RING + LW_EXT
// the long kernel's imaginary-part table runs LONG_TABLE_REACH floats past one period: a detection round's lanes
// read up to 63 x 31 + 5 x 16 = 2,033 floats past its base, a matched-filter pass up to 2 x 956 + 29 = 1,941
// (8 data symbols).  8-symbol frames: 256 + 15,952 + 12 x 12,288 B = 163,664 B of the CU's 163,840
constexpr int LONG_TABLE_REACH = 2048;
constexpr int FRAME_LONG_MIN_CAP = 4100;     // captures longer than this (frames of >= 5 data symbols) run it

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
    for (int i = 0; i < 10; ++i) out[20 - i] = out[i];      // symmetric (the sync kernel folds the taps)
}

}  // namespace ofdm

using namespace ofdm;

#define HIPOK(expr)                                                                             \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return set_error(OFDM_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

static float *wave_re_of(Ctx *c, int len) { return (float *)((char *)c->d_wave + (size_t)len * sizeof(float2) + 64); }

static int ensure_wave(Ctx *c, int conv, int payload) {
    if (conv != OFDM_CONV_C && conv != OFDM_CONV_MATLAB) return set_error(OFDM_E_ARG, "bad conv %d", conv);
    if (payload != OFDM_PAYLOAD_MESSAGE && payload != OFDM_PAYLOAD_TESTER)
        return set_error(OFDM_E_ARG, "frame mode needs a fixed payload (MESSAGE or TESTER), got %d", payload);
    const int key = conv * 4 + payload;      // ofdm_set_message resets the key
    if (c->wave_key == key) return OFDM_OK;
    WaveArgs a{};
    a.n_data = payload_table(payload, c->message, a.table);
    const int len = wave_len_for(a.n_data);
    // [len] float2 waveform | power (64 B) | real parts of one copy (len / FR_REPS floats, 16-B aligned)
    int rc = c->ensure(&c->d_wave, &c->cap_wave, (size_t)len * sizeof(float2) + 64 + (size_t)len / FR_REPS * sizeof(float));
    if (rc) return rc;
    a.wave = (float2 *)c->d_wave;
    a.power = (double *)((char *)c->d_wave + (size_t)len * sizeof(float2));
    rrc_taps(a.taps);
    a.stf_scale = (float)std::sqrt(13.0 / 6.0);
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_C>, dim3(1), dim3(256), 0, c->stream, a);
    else hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_MATLAB>, dim3(1), dim3(256), 0, c->stream, a);
    HIPOK(hipGetLastError());
    // the capture's clean real parts, dense (the sync kernel loads 4 per 16 B instead of 4 complex samples per 32 B)
    HIPOK(hipMemcpy2DAsync(wave_re_of(c, len), sizeof(float), c->d_wave, sizeof(float2), sizeof(float),
                           (size_t)len / FR_REPS, hipMemcpyDeviceToDevice, c->stream));
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
    a.wave_re = wave_re_of(c, c->wave_len);
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
    // the lazy capture's equivalence test runs the same sweep with it switched off (tests/test_gpu_frame.py)
    a.no_lazy = getenv("OFDM_FRAME_NO_LAZY") != nullptr;
    rrc_taps(a.taps);
}

// bits needed for the largest magnitude, as OFDM.c:56-64
static int32_t word_bits(double mn, double mx) {
    const float max_abs = (float)std::fmax(std::fabs(mn), std::fabs(mx));
    return max_abs < 1.0f ? 1 : (int32_t)std::ceil(std::log2((double)max_abs)) + 1;
}

// items per sync -> symbol hand-off: 2^23 items x 1.5 KB (reference message) = 12 GiB of HBM, one launch pair per
// 8M items (A/B, frame mode: 2^18 3.13e8, 2^20 3.33e8, 2^22 3.40e8 symbol-SNR/s; round 6, 2^23 over 2^22: frame
// +0.4 %, frame8 +0.4 %, profiles/r06/frame/ab_chunk.txt -- each pair ends in a tail and K4b' waits for K4b)
#define FRAME_CHUNK_LOG2 23
constexpr int64_t FRAME_CHUNK_ITEMS = int64_t(1) << FRAME_CHUNK_LOG2;
// items per chunk for n_data data symbols: 2^23, capped so that the hand-off buffer holds no more windows than the
// reference message's 2^23 items do (1 + n_data windows of 512 B per item: 12 GiB; ADVICE r3: 8-symbol messages
// would otherwise take 38 GiB)
static int64_t frame_chunk_items(int n_data) {
    return std::min<int64_t>(FRAME_CHUNK_ITEMS, FRAME_CHUNK_ITEMS * 3 / (1 + n_data));
}
constexpr int64_t FRAME_CHUNK_MIN = int64_t(1) << 16;    // halving stops here when the buffer cannot be allocated

// K4b then K4b' over a.n_items items starting at a.item0, through the context's hand-off buffer
static int run_frame_chunk(Ctx *c, FrameArgs &a) {
    const int nw = 1 + a.n_data;
    if (a.n_snr < 1 || a.n_items < 0 || a.n_items + a.n_snr + FRAME_ITEM_RUN > (int64_t(1) << 31))
        return set_error(OFDM_E_ARG, "frame chunk: items or SNR points out of range");
    a.trial0 = a.item0 / a.n_snr;
    a.q0 = (int32_t)(a.item0 % a.n_snr);
    a.snr_magic = 0xFFFFFFFFu / (uint32_t)a.n_snr;
    a.ipb = 4 * (16 / sym_quads(a.n_data));             // whole items per wave (frame_sym_kernel)
    const size_t wbytes = (size_t)((a.n_items + a.ipb - 1) / a.ipb) * a.ipb * nw * 64 * sizeof(float2);
    int rc = c->ensure(&c->d_scratch, &c->cap_scratch, wbytes + (size_t)a.n_items * sizeof(int4) + 256);
    if (rc) return rc;
    a.win = (float2 *)c->d_scratch;
    a.info = (int4 *)((char *)c->d_scratch + ((wbytes + 255) & ~size_t(255)));
    // the capture's imaginary parts: one waveform copy (+ IMT_EXT) for generated captures, the external
    // capture's own for ofdm_receiver
    a.im_period = a.ext ? (1 << 30) : a.wave_len / FR_REPS;
    a.im_magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)a.im_period - 1) / (uint64_t)a.im_period);
    a.imt_len = (a.ext ? a.cap_len : a.im_period) + IMT_EXT;
    const size_t lds = frame_lds_bytes(a.cap_len, a.n_data, a.n_snr, a.imt_len, a.word_stats);
    a.fr_in_cap = fr_in_capture(a.cap_len, a.n_data);
    a.region_floats = wave_region_floats(a.cap_len, a.n_data);
    if (!c->d_work) HIPOK(hipMalloc(&c->d_work, 256));
    a.work = (unsigned long long *)c->d_work;
    HIPOK(hipMemsetAsync(c->d_work, 0, sizeof(unsigned long long), c->stream));
    // one resident grid: every wave starts with a run of items, the rest come from the work counter.  The
    // reference message's sweep (2 data symbols, the default 3008-sample capture, no dumps / word-length
    // statistics) runs the instantiation with that geometry folded in; OFDM_FRAME_GENERIC=1 forces the generic
    // one (the equivalence test)
    const int64_t runs = (a.n_items + FRAME_ITEM_RUN - 1) / FRAME_ITEM_RUN;
    // long captures (frames of >= 5 data symbols): frame_sync_long_kernel keeps one detection round's piece per wave, not
    // the whole capture (3 waves per SIMD instead of 1); sweeps only.  OFDM_FRAME_NO_LONG=1 forces the generic kernel
    // (the equivalence test)
    const bool is_long = a.cap_len > FRAME_LONG_MIN_CAP && a.cap_len - 47 <= 3 * 64 * 31 && !a.ext && !a.dbg_res &&
                         !a.dbg_ints && !a.dbg_bits && !a.dbg_eq && !a.dbg_corr && !a.dbg_frame && !a.word_stats &&
                         2 * fr_len(a.n_data) + 40 <= FRAME_LONG_REGION && !getenv("OFDM_FRAME_NO_LONG") &&
                         !FRAME_STAMPS_BUILD;
    // every capture routed here has Lc > 2 x 64 x 31: the long kernel always runs three detection rounds (its R == 2
    // branches are unreachable; they stay so that the PMC-certified code object does not move)
    static_assert(FRAME_LONG_MIN_CAP - 47 >= 2 * 64 * 31, "long captures take three detection rounds");
    if (is_long) {
        a.region_floats = FRAME_LONG_REGION;
        a.imt_len = a.im_period + LONG_TABLE_REACH;           // the long kernel's wrap-free table
        const size_t lds_l = (size_t)a.n_snr * 2 * 8 + (((size_t)a.imt_len * 4 + 15) & ~size_t(15)) +
                             (size_t)LONG_W * FRAME_LONG_REGION * 4;
        const dim3 gl(occupancy_grid(frame_long_kernel(), 64 * LONG_W, lds_l, c->cus, (runs + LONG_W - 1) / LONG_W, 1));
        launch_frame_long(c->stream, a, gl, lds_l);
        launch_frame_sym(c->stream, a, c->cus);
        HIPOK(hipGetLastError());
        return OFDM_OK;
    }
    const bool fixed = a.n_data == 2 && a.cap_len == cap_len_for(2) && a.wave_len == wave_len_for(2) && !a.ext &&
                       !a.dbg_res && !a.dbg_ints && !a.dbg_bits && !a.dbg_eq && !a.dbg_corr && !a.dbg_frame &&
                       !a.word_stats && !getenv("OFDM_FRAME_GENERIC");
    // Long captures (8-symbol messages: 24 KB per wave) could run one-wave blocks, which fit five per CU where
    // one four-wave block fits; but five waves on four SIMDs leave three SIMDs with one wave each, and
    // the 8-symbol sweep measured 4.07e8 with one-wave blocks against 4.16e8 with four-wave ones (round 4,
    // profiles/r04/ab/h_frame8*.json; after the real-part table 4.28e8 against 4.50e8, and 4.15e8 with two-wave
    // blocks, ae_frame8_blocks.txt).  So one-wave blocks run only when they give every SIMD more waves:
    // resident = whole waves per SIMD x 4, from W x floor(LDS per CU / block LDS), at most 12
    const size_t lds1 = frame_lds_bytes(a.cap_len, a.n_data, a.n_snr, a.imt_len, a.word_stats, 1);
    auto resident = [](size_t b, int w) {
        return std::min<int64_t>(12, w * (int64_t)(FRAME_LDS_PER_CU / b) / 4 * 4);
    };
    const bool one = !fixed && ((resident(lds1, 1) > resident(lds, SYNC_WAVES) && !getenv("OFDM_FRAME_BLOCK4")) ||
                                getenv("OFDM_FRAME_BLOCK1"));
    const void *ks = fixed ? frame_fix_kernel()
                   : one   ? reinterpret_cast<const void *>(&frame_sync_kernel<0, 0, 1>)
                           : reinterpret_cast<const void *>(&frame_sync_kernel<0, 0>);
    const int waves = fixed ? FIX_W : one ? 1 : SYNC_WAVES;
    // the fixed kernel's table: FIX_IMT_COPIES periods (its own layout, see FIX_W)
    const size_t lds_f = frame_lds_bytes(a.cap_len, a.n_data, a.n_snr, FIX_IMT_COPIES * a.im_period + IMT_EXT, 0, FIX_W);
    const dim3 gs(occupancy_grid(ks, 64 * waves, fixed ? lds_f : one ? lds1 : lds, c->cus, (runs + waves - 1) / waves, 1));
    if (fixed) launch_frame_fix(c->stream, a, gs, lds_f);
    else if (one) hipLaunchKernelGGL((frame_sync_kernel<0, 0, 1>), gs, dim3(64), lds1, c->stream, a);
    else hipLaunchKernelGGL((frame_sync_kernel<0, 0>), gs, dim3(SYNC_THREADS), lds, c->stream, a);
    launch_frame_sym(c->stream, a, c->cus);
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
    if (opts->word_stats) {                       // the word-length extremes start at +/- infinity
        std::vector<int64_t> init((size_t)n_snr * OFDM_NCOUNTERS, 0);
        for (int q = 0; q < n_snr; ++q) {
            init[(size_t)q * OFDM_NCOUNTERS + OFDM_C_WL_MIN_Q] = INT64_MAX;
            init[(size_t)q * OFDM_NCOUNTERS + OFDM_C_WL_MAX_Q] = INT64_MIN;
        }
        HIPOK(hipMemcpyAsync(c->d_cnt, init.data(), cbytes, hipMemcpyHostToDevice, c->stream));
    } else {
        HIPOK(hipMemsetAsync(c->d_cnt, 0, cbytes, c->stream));
    }
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
        int64_t chunk = frame_chunk_items(a.n_data);
        for (int64_t i0 = 0; i0 < items;) {
            a.item0 = i0;
            a.n_items = std::min(chunk, items - i0);
            a.add_totals = i0 + a.n_items >= items;
            rc = run_frame_chunk(c, a);
            if (rc == OFDM_E_NOMEM && chunk > FRAME_CHUNK_MIN) {   // nothing launched yet: a smaller buffer
                (void)hipGetLastError();
                chunk /= 2;
                continue;
            }
            if (rc) { c->toc(); return rc; }
            i0 += a.n_items;
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
    if (dp) HIPOK(hipMemcpyAsync(packet_idx, dp, pbytes, hipMemcpyDeviceToHost, c->stream));
    if ((rc = c->read_counters(counters, cbytes))) return rc;     // pinned staging; returns once the copies landed
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
#endif  // OFDM_FRAME_AUX_TU
