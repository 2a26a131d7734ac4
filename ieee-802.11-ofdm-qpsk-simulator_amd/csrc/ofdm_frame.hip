// ofdm_frame.hip -- frame mode: the reference's own trial on gfx950.
//
//   K4a frame_wave_kernel : Transmitter() (OFDM.c:467-618) -- preambles + data symbols, 2x zero
//                           stuffing, 21-tap RRC, x10 repeat, mean power (OFDM.c:637-643).
//   K4b frame_rx_kernel   : one wave per trial: capture (OFDM.c:945-955) + real AWGN (OFDM.c:651),
//                           Packet_Detection (659-683) with sliding sums, Packet_Selection (685-771)
//                           as a wave ballot/min, RRC matched filter evaluated only at the 320+80D
//                           down-sampled instants (965, 984-996), coarse/fine CFO (773-828), then the
//                           same register FFT + LS estimate + demap as symbol mode (830-1165).
//   K4c ota_kernel        : Transmission_Over_Air() on a caller-provided waveform.
//
// The capture lives in LDS (24 KB per wave for the reference's 2-symbol message; frames carry 1..8
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
    uint32_t k0, k1;
    uint32_t table[3 * FR_MAX_DATA];
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
    const Gauss4 g = gauss4(t_lo, t_hi, (uint32_t)b, STREAM_NOISE | q, k0, k1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = 4 * b + j;
        if (k < n) {
            float2 v = x[k];
            v.x = fmaf(sigma, g.z[j], v.x);
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
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

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
    sincospif(2.0f * fr, &s, &c);
    return make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
}

// LDS image of one trial (dynamic shared memory, sized per launch by frame_lds_bytes)
struct FrameLds {
    float2 *r;                  // capture [cap_len]
    float2 *fr;                 // down-sampled frame [fr_len(n_data)]
    unsigned long long *cross;  // Packet_Detection threshold crossings, 1 bit per position
    unsigned long long *acc;    // [n_snr][ACC_SLOTS] per-SNR block accumulators
};
constexpr int ACC_SLOTS = 12;   // 9 counter sums + word-length min / max (q20) + pad
__host__ __device__ inline int cross_words(int cap_len) { return (cap_len - 47 + 63) / 64 + 1; }
__host__ __device__ inline size_t frame_lds_bytes(int cap_len, int n_data, int n_snr) {
    return (size_t)cap_len * 8 + (size_t)fr_len(n_data) * 8 + (size_t)cross_words(cap_len) * 8 +
           (size_t)n_snr * ACC_SLOTS * 8;
}

__global__ __launch_bounds__(64) void frame_rx_kernel(FrameArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int L = a.cap_len, Lc = L - 47;       // Packet_Detection length (OFDM.c:663)
    const int nfr = fr_len(a.n_data);
    FrameLds s;
    s.r = reinterpret_cast<float2 *>(smem);
    s.fr = s.r + L;
    s.cross = reinterpret_cast<unsigned long long *>(s.fr + nfr);
    s.acc = s.cross + cross_words(L);
    float2 *r = s.r, *fr = s.fr;
    unsigned long long *cross = s.cross;
    const int lane = threadIdx.x;
    for (int i = lane; i < a.n_snr * ACC_SLOTS; i += 64) {
        const int k = i % ACC_SLOTS;
        s.acc[i] = k == 10 ? (unsigned long long)INT64_MAX : k == 11 ? (unsigned long long)INT64_MIN : 0ull;
    }
    const int chunk = (Lc + 63) / 64;           // detection positions per lane (< 300: one front each)
    const int64_t items = a.n_trials * a.n_snr;
#ifdef OFDM_FRAME_STAMPS
    unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long stamp_t = __builtin_amdgcn_s_memtime();
#endif
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int q = (int)(it % a.n_snr);
        const int64_t ti = it / a.n_snr;
        const uint64_t t = a.first_trial + (uint64_t)ti;
        const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32), qs = (uint32_t)(a.q_base + q);
        const float sigma = a.sigma[q];
        // ---- capture window (OFDM.c:945-955) + AWGN ----
        int rx_start = a.fixed_start;
        if (rx_start < 0) {
            const uint4 o = philox10(t_lo, t_hi, 0u, STREAM_START | qs, a.k0, a.k1);
            rx_start = (int)(o.x % (uint32_t)(a.wave_len - L));
        }
        if (a.ext && it == 0) {
            for (int n = lane; n < L; n += 64) r[n] = a.ext[n];
        } else {
            const int b0 = rx_start >> 2, b1 = (rx_start + L - 1) >> 2;
            // Gaussian k of the trial's stream goes to waveform sample k (as if Transmission_Over_Air
            // had drawn the whole waveform); only the captured samples are ever evaluated.  Four
            // Philox blocks per lane per pass, their waveform loads issued first.
            for (int bb = b0 + lane; bb <= b1; bb += 256) {
                float2 v[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int k = 4 * (bb + 64 * u) + j;
                        v[u][j] = (bb + 64 * u <= b1 && k < a.wave_len) ? a.wave[k] : make_float2(0.f, 0.f);
                    }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int b = bb + 64 * u;
                    if (b > b1) break;
                    Gauss4 g;
                    if (a.noise == OFDM_NOISE_REAL) g = gauss4(t_lo, t_hi, (uint32_t)b, STREAM_NOISE | qs, a.k0, a.k1);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int n = 4 * b + j - rx_start;
                        if (n >= 0 && n < L) {
                            float2 w = v[u][j];
                            if (a.noise == OFDM_NOISE_REAL) w.x = fmaf(sigma, g.z[j], w.x);   // real-only (D7)
                            r[n] = w;
                        }
                    }
                }
            }
        }
        for (int i = lane; i < cross_words(L); i += 64) cross[i] = 0ull;
        __syncthreads();
        FR_STAMP(0);                                           // capture + noise

        // ---- Word_Optimization_Analysis(Rx_filter_signal) (OFDM.c:38-73, 962-967): the full RRC
        // matched filter of the capture, min / max over real and imaginary parts (opt-in) ----
        if (a.word_stats) {
            float mn = 1e9f, mx = -1e9f;
            for (int k = lane; k < L + 20; k += 64) {
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
            if (lane == 0) {
                unsigned long long *sl = s.acc + q * ACC_SLOTS;
                sl[10] = (unsigned long long)min((long long)sl[10], (long long)__float2ll_rn(mn * (float)OFDM_EVM_Q_SCALE));
                sl[11] = (unsigned long long)max((long long)sl[11], (long long)__float2ll_rn(mx * (float)OFDM_EVM_Q_SCALE));
            }
        }

        // ---- Packet_Detection (OFDM.c:659-683): M[n] = |sum r[n+k] r[n+k+16]|^2 / (sum |r[n+k+16]|^2)^2,
        // k < 32, no conjugate, on the UNFILTERED capture; sliding sums over each lane's chunk with the
        // LDS reads issued 8 positions at a time.  M > 0.75 (OFDM.c:687, 695) is tested as
        // num > 0.75 den, which keeps the division's 0/0 -> false and x/0 -> true outcomes. ----
        const int n0 = lane * chunk, n1 = min(n0 + chunk, Lc);
        int first = -1, last = -1;                  // first / last crossing in this lane's chunk
        if (n0 < n1) {
            float sx = 0.f, sy = 0.f, pw = 0.f;
#pragma unroll 8
            for (int k = 0; k < 32; ++k) {
                const float2 u = r[n0 + k], v = r[n0 + k + 16];
                sx += u.x * v.x - u.y * v.y;
                sy += u.x * v.y + u.y * v.x;
                pw += v.x * v.x + v.y * v.y;
            }
            unsigned long long word = 0ull;
            for (int nb = n0; nb < n1; nb += 8) {
                float2 o0[8], o1[8], i0[8], i1[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {           // reads past the capture land in fr/cross: unused
                    o0[k] = r[nb + k]; o1[k] = r[nb + k + 16]; i0[k] = r[nb + k + 32]; i1[k] = r[nb + k + 48];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int n = nb + k;
                    if (n >= n1) break;
                    const float num = sx * sx + sy * sy, den = pw * pw;
                    if (a.dbg_corr && it == 0) a.dbg_corr[n] = num / den;
                    if (num > 0.75f * den) {
                        word |= 1ull << (n & 63);
                        if (first < 0) first = n;
                        last = n;
                    }
                    if ((n & 63) == 63 || n + 1 == n1) {
                        if (word) atomicOr(&cross[n >> 6], word);
                        word = 0ull;
                    }
                    sx += (i0[k].x * i1[k].x - i0[k].y * i1[k].y) - (o0[k].x * o1[k].x - o0[k].y * o1[k].y);
                    sy += (i0[k].x * i1[k].y + i0[k].y * i1[k].x) - (o0[k].x * o1[k].y + o0[k].y * o1[k].x);
                    pw += (i1[k].x * i1[k].x + i1[k].y * i1[k].y) - (o1[k].x * o1[k].x + o1[k].y * o1[k].y);
                }
            }
        }

        // ---- Packet_Selection (OFDM.c:685-771): crossing idx[j] is a front iff idx[j] - idx[j-1] > 300
        // (idx[-1] = -1).  Fronts are > 300 apart and a chunk is < 300 positions, so only a lane's
        // first crossing can be one, and its predecessor is the last crossing of the earlier chunks:
        // an exclusive prefix max over lanes.  The first front x with a later front and
        // M[front+230] > 0.75 gives packet_idx = front + len_RRC_rx + 1; otherwise 0 (OFDM.c:752-761). ----
        int pm = last;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(pm, o, 64);
            if (lane >= o) pm = max(pm, t);
        }
        int prev = __shfl_up(pm, 1, 64);
        if (lane == 0) prev = -1;
        const int front = (first >= 0 && first - prev > 300) ? first : -1;
        __syncthreads();                            // every crossing word is in LDS
        FR_STAMP(1);                                           // packet detection
        const bool valid = front >= 0 && front + 230 < Lc && bit_at(cross, front + 230);
        const int maxf = wave_max_i(front);
        const int cand = wave_min_i((valid && front < maxf) ? front : 0x7fffffff);
        const bool sync_fail = cand == 0x7fffffff;
        const int p = sync_fail ? 0 : cand + 10 + 1;           // len_RRC_rx + 1 (OFDM.c:758)
        FR_STAMP(2);                                           // packet selection

        // ---- RRC matched filter at the down-sampled instants p + 2i (OFDM.c:965, 992-996): a lane
        // takes 8 consecutive outputs, i.e. one 35-sample window of the capture held in registers ----
        bool oob_l = false;
        for (int ib = 8 * lane; ib < nfr; ib += 512) {
            const int nb = p + 2 * ib - 20;             // first capture sample the 8 outputs touch
            float2 win[35];
#pragma unroll
            for (int k = 0; k < 35; ++k) {
                const int m = nb + k;
                win[k] = (m >= 0 && m < L) ? r[m] : make_float2(0.f, 0.f);   // Convolution zero-pads
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = ib + t;
                if (i >= nfr) break;
                float2 v = make_float2(0.f, 0.f);
                if (p + 2 * i >= L + 20) {
                    oob_l = true;                                // the reference reads past its buffer
                } else {
#pragma unroll
                    for (int j = 0; j < 21; ++j) {
                        const float2 x = win[2 * t + 20 - j];
                        v.x = fmaf(x.x, a.taps[j], v.x);
                        v.y = fmaf(x.y, a.taps[j], v.y);
                    }
                }
                fr[i] = v;
            }
        }
        const bool oob = __any(oob_l);
        __syncthreads();
        FR_STAMP(3);                                           // matched filter + down-sample

        // ---- Coarse CFO (OFDM.c:773-804): 16-lag autocorrelation of the short preamble ----
        float px = 0.f, py = 0.f;
        if (lane < 16) { const float2 u = fr[80 + lane], v = fr[96 + lane]; px = u.x * v.x + u.y * v.y; py = u.y * v.x - u.x * v.y; }
        px = wave_sum_f(px); py = wave_sum_f(py);
        double fc = (-1.0 / (2.0 * M_PI * 16.0 * TS)) * (double)atan2f(py, px);
        if (a.float_cfo) fc = (double)(float)fc;
        for (int i = lane; i < nfr; i += 64) fr[i] = cfo_rot(fr[i], fc * TS, i);
        __syncthreads();
        // ---- Fine CFO (OFDM.c:806-828): 64-lag over the two long training symbols ----
        {
            const float2 u = fr[192 + lane], v = fr[256 + lane];
            px = wave_sum_f(u.x * v.x + u.y * v.y);
            py = wave_sum_f(u.y * v.x - u.x * v.y);
        }
        double ff = (-1.0 / (2.0 * M_PI * 64.0 * TS)) * (double)atan2f(py, px);
        if (a.float_cfo) ff = (double)(float)ff;
        __syncthreads();
        for (int i = lane; i < nfr; i += 64) fr[i] = cfo_rot(fr[i], ff * TS, i);
        __syncthreads();
        if (a.dbg_frame && it == 0) for (int i = lane; i < nfr; i += 64) a.dbg_frame[i] = fr[i];
        FR_STAMP(4);                                           // coarse + fine CFO

        // ---- LS estimate + CP strip + fft + ZF + slicer + demap (OFDM.c:830-1100).  Quad k carries
        // {LTF1, LTF2, D_2k, D_2k+1}: the estimate is formed inside each quad (two broadcasts) ----
        const int role = lane & 3;
        const int dsym = 2 * (lane >> 2) + (role & 1);
        const bool dlane = role >= 2 && dsym < a.n_data;
        const int dsc = min(dsym, a.n_data - 1);
        const int w0 = role == 0 ? 192 : role == 1 ? 256 : 336 + 80 * dsc;
        float2 x[64];
        static_for<0, 64>([&](auto nc) {
            constexpr int n = decltype(nc)::value;
            const float2 v = fr[w0 + n];
            x[n] = (n & 1) ? make_float2(-v.x, -v.y) : v;        // fft() = DFT(x (-1)^n)
        });
#ifndef OFDM_FRAME_NO_FFT   // profiling switch: time the sync phases alone
        fft64<false>(x);
#endif
        const uint32_t w[3] = {a.table[3 * dsc], a.table[3 * dsc + 1], a.table[3 * dsc + 2]};
        SymState st;
        sym_init(st);
        const bool dump = a.dbg_eq && it == 0 && dlane;
        float2 *deq = dump ? a.dbg_eq + 48 * dsym : nullptr;
        auto Hof = [&](float2 Y, auto binc) { return ls_equalise<decltype(binc)::value>(Y); };
#ifndef OFDM_FRAME_NO_FFT
        static_for<0, 4>([&](auto rc) { demap_sub<true, decltype(rc)::value, 2>(x, w, Hof, deq, st); });
#else
        st.evm_pre = x[5].x;
#endif
        FR_STAMP(5);                                           // FFT + LS + demap
        const float fe = wave_sum_f(dlane ? finish_evm<2>(st) : 0.f);
        const uint32_t ferr = wave_sum_u32(dlane ? st.be : 0u), fax = wave_sum_u32(dlane ? st.ax : 0u);
        if (lane == 0) {
            unsigned long long *sl = s.acc + q * ACC_SLOTS;
            sl[0] += ferr;
            sl[1] += ferr > 0u;
            sl[2] += fax;
            sl[3] += sync_fail;
            sl[4] += oob;
            const float N = 48.0f * (float)a.n_data;
            sl[5] += (unsigned long long)(int64_t)__float2ll_rn(fe * (float)OFDM_EVM_Q_SCALE);
            const float db = fe > 0.f ? fmaxf(3.01029995663981195214f * __builtin_amdgcn_logf(fe / N), -400.f) : -400.f;
            sl[6] += (unsigned long long)(int64_t)__float2ll_rn(db * (float)OFDM_EVM_Q_SCALE);
            float dbp = -INFINITY;
            if (fax > 0u) {
                dbp = 3.01029995663981195214f * __builtin_amdgcn_logf(2.0f * (float)fax / N);
                sl[7] += (unsigned long long)(int64_t)__float2ll_rn(dbp * (float)OFDM_EVM_Q_SCALE);
                sl[8] += 1ull;
            }
            if (a.pidx_out) a.pidx_out[(int64_t)q * a.n_trials + ti] = p;
            if (it == 0) {
                if (a.dbg_res) { a.dbg_res[0] = db; a.dbg_res[1] = dbp; a.dbg_res[2] = (float)ferr / (96.0f * a.n_data); }
                if (a.dbg_ints) { a.dbg_ints[0] = p; a.dbg_ints[1] = sync_fail; a.dbg_ints[2] = oob; a.dbg_ints[3] = rx_start; }
            }
        }
        if (it == 0 && a.dbg_bits && dlane) {
            a.dbg_bits[3 * dsym] = st.d[0]; a.dbg_bits[3 * dsym + 1] = st.d[1]; a.dbg_bits[3 * dsym + 2] = st.d[2];
        }
        __syncthreads();
        FR_STAMP(6);                                           // counters
    }
#ifdef OFDM_FRAME_STAMPS
    if (threadIdx.x == 0 && a.stamps)
        for (int k = 0; k < 7; ++k) atomicAdd(&a.stamps[k], stamp_acc[k]);
#endif
    __syncthreads();
    for (int i = lane; i < a.n_snr * 9; i += 64) {
        const int q = i / 9, k = i % 9;
        const unsigned long long v = s.acc[q * ACC_SLOTS + k];
        if (!v) continue;
        const int c = k == 0 ? OFDM_C_BIT_ERR : k == 1 ? OFDM_C_FRAME_ERR : k == 2 ? OFDM_C_EVM_POST_AXIS
                    : k == 3 ? OFDM_C_SYNC_FAIL : k == 4 ? OFDM_C_OOB : k == 5 ? OFDM_C_EVM_PRE_Q
                    : k == 6 ? OFDM_C_EVMDB_PRE_Q : k == 7 ? OFDM_C_EVMDB_POST_Q : OFDM_C_EVMDB_POST_FINITE;
        atomicAdd(&a.counters[q * OFDM_NCOUNTERS + c], v);
    }
    if (a.word_stats) {
        for (int q = lane; q < a.n_snr; q += 64) {
            long long *c = reinterpret_cast<long long *>(a.counters + q * OFDM_NCOUNTERS);
            atomicMin(&c[OFDM_C_WL_MIN_Q], (long long)s.acc[q * ACC_SLOTS + 10]);
            atomicMax(&c[OFDM_C_WL_MAX_Q], (long long)s.acc[q * ACC_SLOTS + 11]);
        }
    }
    if (blockIdx.x == 0) {
        for (int q = lane; q < a.n_snr; q += 64) {
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
    a.word_stats = o->word_stats ? 1 : 0;
    rrc_taps(a.taps);
}

// bits needed for the largest magnitude, as OFDM.c:56-64
static int32_t word_bits(double mn, double mx) {
    const float max_abs = (float)std::fmax(std::fabs(mn), std::fabs(mx));
    return max_abs < 1.0f ? 1 : (int32_t)std::ceil(std::log2((double)max_abs)) + 1;
}

static unsigned frame_grid(Ctx *c, int64_t items, size_t lds) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&frame_rx_kernel), 64,
                                                     lds) != hipSuccess || per_cu < 1)
        per_cu = 2;
    const int64_t cap = (int64_t)per_cu * c->cus * 4;
    return (unsigned)std::max<int64_t>(1, std::min(items, cap));
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
    const size_t lds = frame_lds_bytes(L, nd, 1);
    c->tic(Ctx::K_FRAME);
    hipLaunchKernelGGL(frame_rx_kernel, dim3(1), dim3(64), lds, c->stream, a);
    c->toc();
    HIPOK(hipGetLastError());
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
        const size_t lds = frame_lds_bytes(a.cap_len, a.n_data, a.n_snr);
#ifdef OFDM_FRAME_STAMPS
        unsigned long long *dst = nullptr;
        HIPOK(hipMalloc(&dst, 64));
        HIPOK(hipMemset(dst, 0, 64));
        a.stamps = dst;
#endif
        c->tic(Ctx::K_FRAME);
        hipLaunchKernelGGL(frame_rx_kernel, dim3(frame_grid(c, n_trials * a.n_snr, lds)), dim3(64), lds, c->stream, a);
        c->toc();
        HIPOK(hipGetLastError());
#ifdef OFDM_FRAME_STAMPS
        unsigned long long hs[8];
        HIPOK(hipMemcpy(hs, dst, 64, hipMemcpyDeviceToHost));
        hipFree(dst);
        static const char *names[7] = {"capture+noise", "detection", "selection", "matched filter", "cfo",
                                       "fft+ls+demap", "counters"};
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
