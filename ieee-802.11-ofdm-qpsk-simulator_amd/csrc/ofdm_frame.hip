// ofdm_frame.hip -- frame mode: the reference's own trial on gfx950.
//
//   K4a frame_wave_kernel : Transmitter() (OFDM.c:467-618) -- preambles + data symbols, 2x zero
//                           stuffing, 21-tap RRC, x10 repeat, mean power (OFDM.c:637-643).
//   K4b frame_rx_kernel   : one wave per trial: capture (OFDM.c:945-955) + real AWGN (OFDM.c:651),
//                           Packet_Detection (659-683) with sliding sums, Packet_Selection (685-771)
//                           as a wave ballot/min, RRC matched filter evaluated only at the 480
//                           down-sampled instants (965, 984-996), coarse/fine CFO (773-828), then the
//                           same register FFT + LS estimate + demap as symbol mode (830-1165).
//   K4c ota_kernel        : Transmission_Over_Air() on a caller-provided waveform.
//
// The capture lives in LDS (24 KB per wave); detection keeps only the >0.75 crossings as a bit
// mask, since Packet_Selection needs nothing else (it re-reads Corr_Out only at front+230).
#include "ofdm_internal.h"
#include "ofdm_rxcommon.h"
#include "ofdm_ctx.h"
#include <cmath>
#include <cstring>
#include <vector>

namespace ofdm {

constexpr int FR_SAMPLES = 480;              // 160 STF + 160 LTF + 2 x 80 data (OFDM.c:569)
constexpr int FR_OS = 2 * FR_SAMPLES;        // 2x zero-stuffed (OFDM.c:587-595)
constexpr int FR_FILT = FR_OS + 20;          // + 20 RRC tail (OFDM.c:603-605)
constexpr int FR_REPS = 10;                  // OFDM.c:607-612
constexpr int WAVE_LEN = FR_FILT * FR_REPS;  // 9800
constexpr int CAP_MAX = 3008;                // floor(0.307 * 9800) (OFDM.c:945)
constexpr int CHUNK = 47;                    // detection positions per lane: ceil(2961 / 64)
constexpr double TS = 1.0 / 20e6;            // OFDM.c:16-17

// short training tones S_k at bins 6..58 (OFDM.c:483-490): +-1 on every 4th tone, times (1+j)
__host__ __device__ constexpr int stf_sign(int bin) {
    constexpr int8_t S[53] = {0, 0, 1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 0,
                              0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0};
    return (bin >= 6 && bin <= 58) ? S[bin - 6] : 0;
}

struct WaveArgs {
    float2 *wave;        // [WAVE_LEN]
    double *power;       // mean |x|^2 over the waveform
    uint32_t table[6];   // payload words of the 2 data symbols
    float taps[21];
    float stf_scale;     // sqrt(13/6) as the float of OFDM.c:479
};

struct FrameArgs {
    const float2 *wave;        // repeated frame waveform (K4a or caller data)
    const float2 *ext;         // external capture (ofdm_receiver), used for item 0 when non-null
    uint64_t first_trial;
    int64_t n_trials;
    int32_t n_snr, q_base;
    int32_t cap_len, float_cfo, matlab, fixed_start, noise, wave_len;
    uint32_t k0, k1;
    uint32_t table[6];
    unsigned long long *counters;   // [n_snr][OFDM_NCOUNTERS]
    int32_t *pidx_out;              // [n_snr][n_trials] or null
    // per-trial debug outputs of item 0 (ofdm_receiver), all optional
    float *dbg_res;                 // EVM_dB pre, EVM_dB post, BER
    int32_t *dbg_ints;              // packet_idx, sync_fail, oob, rx_start
    uint32_t *dbg_bits;             // 6 words (2 symbols x 96 bits, MSB first)
    float2 *dbg_eq;                 // 2 x 48 equalised subcarriers
    float *dbg_corr;                // Corr_Out (cap_len - 47)
    float2 *dbg_frame;              // 480 samples after fine CFO
    float taps[21];
    float sigma[OFDM_MAX_SNR];
};

// ======================================================================== K4a: waveform
template <int CONV>
__global__ __launch_bounds__(256) void frame_wave_kernel(WaveArgs a) {
    __shared__ float2 T[4][64];          // STF, LTF, D0, D1 time symbols
    __shared__ float2 fr[FR_SAMPLES];
    __shared__ double red[256];
    const int tid = threadIdx.x;
    if (tid < 4) {
        const uint32_t w[3] = {a.table[3 * (tid & 1)], a.table[3 * (tid & 1) + 1], a.table[3 * (tid & 1) + 2]};
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
    // frame = [S(160) L(160) D1(80) D2(80)] (OFDM.c:569-583); short = first 16 samples x10,
    // long = [T(32:64) T T] (Preamble_Generator, OFDM.c:392-398), data = [x(48:64) x] (559-565)
    for (int n = tid; n < FR_SAMPLES; n += blockDim.x) {
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
    for (int k = tid; k < FR_FILT; k += blockDim.x) {
        // Convolution(oversampled frame, RRC) (OFDM.c:342-364); odd taps of the zero-stuffed input vanish
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 21; ++j) {
            const int m = k - j;
            if (m >= 0 && m < FR_OS && !(m & 1)) {
                const float2 x = fr[m >> 1];
                acc.x = fmaf(a.taps[j], x.x, acc.x);
                acc.y = fmaf(a.taps[j], x.y, acc.y);
            }
        }
        for (int r = 0; r < FR_REPS; ++r) a.wave[k + r * FR_FILT] = acc;
        pw += (double)acc.x * acc.x + (double)acc.y * acc.y;
    }
    red[tid] = pw;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    if (tid == 0) *a.power = red[0] / FR_FILT;    // mean over 10 identical repeats
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

struct FrSlots { unsigned long long v[10]; };   // per-SNR block accumulators

__global__ __launch_bounds__(64) void frame_rx_kernel(FrameArgs a) {
    __shared__ float2 r[CAP_MAX];
    __shared__ float2 fr[FR_SAMPLES];
    __shared__ unsigned long long cross[48];
    __shared__ unsigned long long acc[OFDM_MAX_SNR][10];
    const int lane = threadIdx.x;
    for (int i = lane; i < a.n_snr * 10; i += 64) (&acc[0][0])[i] = 0ull;
    const int L = a.cap_len, Lc = L - 47;       // Packet_Detection length (OFDM.c:663)
    const int64_t items = a.n_trials * a.n_snr;
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
            // had drawn all 9800); only the captured samples are ever evaluated
            for (int b = b0 + lane; b <= b1; b += 64) {
                Gauss4 g;
                if (a.noise == OFDM_NOISE_REAL) g = gauss4(t_lo, t_hi, (uint32_t)b, STREAM_NOISE | qs, a.k0, a.k1);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int n = 4 * b + j - rx_start;
                    if (n >= 0 && n < L) {
                        float2 v = a.wave[4 * b + j];
                        if (a.noise == OFDM_NOISE_REAL) v.x = fmaf(sigma, g.z[j], v.x);   // real-only (D7)
                        r[n] = v;
                    }
                }
            }
        }
        if (lane < 48) cross[lane] = 0ull;
        __syncthreads();

        // ---- Packet_Detection (OFDM.c:659-683): M[n] = |sum r[n+k] r[n+k+16]|^2 / (sum |r[n+k+16]|^2)^2,
        // k < 32, no conjugate, on the UNFILTERED capture; sliding sums over each lane's chunk ----
        const int n0 = lane * CHUNK, n1 = min(n0 + CHUNK, Lc);
        unsigned long long mask = 0ull;
        if (n0 < n1) {
            float sx = 0.f, sy = 0.f, pw = 0.f;
            for (int k = 0; k < 32; ++k) {
                const float2 u = r[n0 + k], v = r[n0 + k + 16];
                sx += u.x * v.x - u.y * v.y;
                sy += u.x * v.y + u.y * v.x;
                pw += v.x * v.x + v.y * v.y;
            }
            for (int n = n0; n < n1; ++n) {
                const float M = (sx * sx + sy * sy) / (pw * pw);
                if (M > 0.75f) mask |= 1ull << (n - n0);          // Packet_Selection threshold (OFDM.c:687)
                if (a.dbg_corr && it == 0) a.dbg_corr[n] = M;
                if (n + 1 < n1) {
                    const float2 o0 = r[n], o1 = r[n + 16], i0 = r[n + 32], i1 = r[n + 48];
                    sx += (i0.x * i1.x - i0.y * i1.y) - (o0.x * o1.x - o0.y * o1.y);
                    sy += (i0.x * i1.y + i0.y * i1.x) - (o0.x * o1.y + o0.y * o1.x);
                    pw += (i1.x * i1.x + i1.y * i1.y) - (o1.x * o1.x + o1.y * o1.y);
                }
            }
            atomicOr(&cross[n0 >> 6], mask << (n0 & 63));
            if ((n0 & 63) + CHUNK > 64) atomicOr(&cross[(n0 >> 6) + 1], mask >> (64 - (n0 & 63)));
        }
        __syncthreads();

        // ---- Packet_Selection (OFDM.c:685-771): a crossing i is a front iff i - prev > 300 with
        // prev = previous crossing or -1, i.e. i >= 300 and no crossing in [i-300, i-1]; the first
        // front x with a later front and M[front+230] > 0.75 gives packet_idx = front + 11.  Fronts
        // are > 300 apart, so a lane's 47-wide chunk holds at most one. ----
        int front = -1;
        for (unsigned long long m = mask; m; m &= m - 1) {
            const int i = n0 + __builtin_ctzll(m);
            if (i >= 300 && !(i >= 1 && bit_at(cross, i - 1)) && !any_bits(cross, i - 300, i - 1)) { front = i; break; }
        }
        const bool valid = front >= 0 && front + 230 < Lc && bit_at(cross, front + 230);
        const int maxf = wave_max_i(front);
        const int cand = wave_min_i((valid && front < maxf) ? front : 0x7fffffff);
        const bool sync_fail = cand == 0x7fffffff;
        const int p = sync_fail ? 0 : cand + 10 + 1;           // len_RRC_rx + 1 (OFDM.c:758)

        // ---- RRC matched filter at the down-sampled instants p + 2i (OFDM.c:965, 992-996) ----
        bool oob_l = false;
        for (int i = lane; i < FR_SAMPLES; i += 64) {
            const int n = p + 2 * i;
            float2 v = make_float2(0.f, 0.f);
            if (n >= L + 20) {
                oob_l = true;                                    // the reference reads past its buffer
            } else {
#pragma unroll
                for (int j = 0; j < 21; ++j) {
                    const int m = n - j;
                    if (m >= 0 && m < L) {
                        const float2 x = r[m];
                        v.x = fmaf(x.x, a.taps[j], v.x);
                        v.y = fmaf(x.y, a.taps[j], v.y);
                    }
                }
            }
            fr[i] = v;
        }
        const bool oob = __any(oob_l);
        __syncthreads();

        // ---- Coarse CFO (OFDM.c:773-804): 16-lag autocorrelation of the short preamble ----
        float px = 0.f, py = 0.f;
        if (lane < 16) { const float2 u = fr[80 + lane], v = fr[96 + lane]; px = u.x * v.x + u.y * v.y; py = u.y * v.x - u.x * v.y; }
        px = wave_sum_f(px); py = wave_sum_f(py);
        double fc = (-1.0 / (2.0 * M_PI * 16.0 * TS)) * (double)atan2f(py, px);
        if (a.float_cfo) fc = (double)(float)fc;
        for (int i = lane; i < FR_SAMPLES; i += 64) fr[i] = cfo_rot(fr[i], fc * TS, i);
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
        for (int i = lane; i < FR_SAMPLES; i += 64) fr[i] = cfo_rot(fr[i], ff * TS, i);
        __syncthreads();
        if (a.dbg_frame && it == 0) for (int i = lane; i < FR_SAMPLES; i += 64) a.dbg_frame[i] = fr[i];

        // ---- LS estimate + CP strip + fft + ZF + slicer + demap (OFDM.c:830-1100); every quad
        // computes the same 4 windows {LTF1, LTF2, D0, D1}, quad 0 reports ----
        const int role = lane & 3;
        const int w0 = role == 0 ? 192 : role == 1 ? 256 : (role == 2 ? 336 : 416);
        float2 x[64];
        static_for<0, 64>([&](auto nc) {
            constexpr int n = decltype(nc)::value;
            const float2 v = fr[w0 + n];
            x[n] = (n & 1) ? make_float2(-v.x, -v.y) : v;        // fft() = DFT(x (-1)^n)
        });
        fft64<false>(x);
        const uint32_t w[3] = {a.table[3 * (role & 1)], a.table[3 * (role & 1) + 1], a.table[3 * (role & 1) + 2]};
        SymState st;
        sym_init(st);
        const bool dump = a.dbg_eq && it == 0 && lane < 4 && role >= 2;
        float2 *deq = dump ? a.dbg_eq + 48 * (role - 2) : nullptr;
        auto Hof = [&](float2 Y, auto binc) { return ls_equalise<decltype(binc)::value>(Y); };
        static_for<0, 4>([&](auto rc) { demap_sub<true, decltype(rc)::value, 2>(x, w, Hof, deq, st); });
        const uint32_t be = st.be, ax = st.ax;
        const float evm = finish_evm<2>(st);
        const float e_other = dpp_f<0xB1>(evm);
        const uint32_t be_other = dpp_u<0xB1>(be), ax_other = dpp_u<0xB1>(ax);
        if (lane == 2) {
            const float fe = evm + e_other;
            const uint32_t ferr = be + be_other, fax = ax + ax_other;
            unsigned long long *s = acc[q];
            s[0] += ferr;
            s[1] += ferr > 0u;
            s[2] += fax;
            s[3] += sync_fail;
            s[4] += oob;
            const float N = 96.0f;
            s[5] += (unsigned long long)(int64_t)__float2ll_rn(fe * (float)OFDM_EVM_Q_SCALE);
            const float db = fe > 0.f ? fmaxf(3.01029995663981195214f * __builtin_amdgcn_logf(fe / N), -400.f) : -400.f;
            s[6] += (unsigned long long)(int64_t)__float2ll_rn(db * (float)OFDM_EVM_Q_SCALE);
            float dbp = -INFINITY;
            if (fax > 0u) {
                dbp = 3.01029995663981195214f * __builtin_amdgcn_logf(2.0f * (float)fax / N);
                s[7] += (unsigned long long)(int64_t)__float2ll_rn(dbp * (float)OFDM_EVM_Q_SCALE);
                s[8] += 1ull;
            }
            if (a.pidx_out) a.pidx_out[(int64_t)q * a.n_trials + ti] = p;
            if (it == 0) {
                if (a.dbg_res) { a.dbg_res[0] = db; a.dbg_res[1] = dbp; a.dbg_res[2] = (float)ferr / 192.0f; }
                if (a.dbg_ints) { a.dbg_ints[0] = p; a.dbg_ints[1] = sync_fail; a.dbg_ints[2] = oob; a.dbg_ints[3] = rx_start; }
            }
        }
        if (it == 0 && a.dbg_bits && lane >= 2 && lane < 4) {
            a.dbg_bits[3 * (lane - 2)] = st.d[0]; a.dbg_bits[3 * (lane - 2) + 1] = st.d[1]; a.dbg_bits[3 * (lane - 2) + 2] = st.d[2];
        }
        __syncthreads();
    }
    __syncthreads();
    for (int i = lane; i < a.n_snr * 9; i += 64) {
        const int q = i / 9, k = i % 9;
        const unsigned long long v = acc[q][k];
        if (!v) continue;
        const int c = k == 0 ? OFDM_C_BIT_ERR : k == 1 ? OFDM_C_FRAME_ERR : k == 2 ? OFDM_C_EVM_POST_AXIS
                    : k == 3 ? OFDM_C_SYNC_FAIL : k == 4 ? OFDM_C_OOB : k == 5 ? OFDM_C_EVM_PRE_Q
                    : k == 6 ? OFDM_C_EVMDB_PRE_Q : k == 7 ? OFDM_C_EVMDB_POST_Q : OFDM_C_EVMDB_POST_FINITE;
        atomicAdd(&a.counters[q * OFDM_NCOUNTERS + c], v);
    }
    if (blockIdx.x == 0) {
        for (int q = lane; q < a.n_snr; q += 64) {
            unsigned long long *c = a.counters + q * OFDM_NCOUNTERS;
            atomicAdd(&c[OFDM_C_FRAMES], (unsigned long long)a.n_trials);
            atomicAdd(&c[OFDM_C_SYMBOLS], (unsigned long long)(2 * a.n_trials));
            atomicAdd(&c[OFDM_C_BITS], (unsigned long long)(192 * a.n_trials));
            atomicAdd(&c[OFDM_C_EVM_TERMS], (unsigned long long)(96 * a.n_trials));
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
    const int key = conv * 4 + payload;
    if (c->wave_key == key) return OFDM_OK;
    int rc = c->ensure(&c->d_wave, &c->cap_wave, WAVE_LEN * sizeof(float2) + 64);
    if (rc) return rc;
    WaveArgs a{};
    a.wave = (float2 *)c->d_wave;
    a.power = (double *)((char *)c->d_wave + WAVE_LEN * sizeof(float2));
    payload_table(payload, a.table);
    rrc_taps(a.taps);
    a.stf_scale = (float)std::sqrt(13.0 / 6.0);
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_C>, dim3(1), dim3(256), 0, c->stream, a);
    else hipLaunchKernelGGL(frame_wave_kernel<OFDM_CONV_MATLAB>, dim3(1), dim3(256), 0, c->stream, a);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(&c->wave_power, a.power, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    c->wave_key = key;
    c->wave_len = WAVE_LEN;
    return OFDM_OK;
}

static int check_opts(const ofdm_rx_opts *o) {
    if (!o) return set_error(OFDM_E_ARG, "opts is NULL");
    if (o->cap_len < 400 || o->cap_len > CAP_MAX) return set_error(OFDM_E_ARG, "cap_len must be in [400, %d]", CAP_MAX);
    if (o->fixed_start > WAVE_LEN - o->cap_len) return set_error(OFDM_E_ARG, "fixed_start beyond the waveform");
    return OFDM_OK;
}

static void fill_frame_args(FrameArgs &a, Ctx *c, const ofdm_rx_opts *o, int noise, uint64_t seed, int payload) {
    a.wave = (const float2 *)c->d_wave;
    a.cap_len = o->cap_len;
    a.float_cfo = o->float_cfo;
    a.matlab = o->matlab_slicer;
    a.fixed_start = o->fixed_start;
    a.noise = noise;
    a.wave_len = WAVE_LEN;
    a.k0 = (uint32_t)seed;
    a.k1 = (uint32_t)(seed >> 32);
    payload_table(payload, a.table);
    rrc_taps(a.taps);
}

static unsigned frame_grid(Ctx *c, int64_t items) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&frame_rx_kernel), 64, 0) !=
            hipSuccess || per_cu < 1)
        per_cu = 4;
    const int64_t cap = (int64_t)per_cu * c->cus * 4;
    return (unsigned)std::max<int64_t>(1, std::min(items, cap));
}

extern "C" {

int ofdm_transmitter(ofdm_ctx *ctx, int conv, int payload, int float_taps, float *tx_out, int32_t max_complex,
                     int32_t *len_out) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    (void)float_taps;   // taps are fp32 on the GPU either way (OFDM.c:32 values)
    if (!c || !tx_out || !len_out) return set_error(OFDM_E_ARG, "bad transmitter arguments");
    if (max_complex < WAVE_LEN) return set_error(OFDM_E_ARG, "tx_out needs %d complex samples", WAVE_LEN);
    HIPOK(hipSetDevice(c->device));
    int rc = ensure_wave(c, conv, payload);
    if (rc) return rc;
    HIPOK(hipMemcpyAsync(tx_out, c->d_wave, WAVE_LEN * sizeof(float2), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    *len_out = WAVE_LEN;
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
    int rc = check_opts(opts);
    if (rc) return rc;
    HIPOK(hipSetDevice(c->device));
    if ((rc = ensure_wave(c, OFDM_CONV_C, payload))) return rc;
    const int L = opts->cap_len;
    // scratch: capture | counters | res | ints | bits | eq
    const size_t off_cnt = ((size_t)L * sizeof(float2) + 255) & ~size_t(255);
    const size_t off_res = off_cnt + OFDM_NCOUNTERS * 8, off_int = off_res + 16, off_bits = off_int + 16;
    const size_t off_eq = off_bits + 32, total = off_eq + 96 * sizeof(float2);
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
    c->tic(Ctx::K_FRAME);
    hipLaunchKernelGGL(frame_rx_kernel, dim3(1), dim3(64), 0, c->stream, a);
    c->toc();
    HIPOK(hipGetLastError());
    float res[4];
    int32_t ints[4];
    uint32_t words[8];
    float2 eq[96];
    HIPOK(hipMemcpyAsync(res, base + off_res, 16, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(ints, base + off_int, 16, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(words, base + off_bits, 32, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(eq, base + off_eq, sizeof(eq), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    if (res3) { res3[0] = res[0]; res3[1] = res[1]; res3[2] = res[2]; }
    if (ints4) { ints4[0] = ints[0]; ints4[1] = ints[1]; ints4[2] = ints[2]; ints4[3] = 0; }
    if (bits_out)
        for (int b = 0; b < 192; ++b) bits_out[b] = (int32_t)((words[b / 32] >> (31 - (b & 31))) & 1u);
    if (eq_out) std::memcpy(eq_out, eq, sizeof(eq));
    return OFDM_OK;
}

int ofdm_frame_sweep(ofdm_ctx *ctx, const ofdm_cfg *cfg, const ofdm_rx_opts *opts, const double *snr_db, int n_snr,
                     uint64_t first_trial, int64_t n_trials, int64_t *counters, int32_t *packet_idx) {
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    if (!c) return set_error(OFDM_E_ARG, "ctx is NULL");
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if ((rc = check_opts(opts))) return rc;
    if (n_snr < 0 || (n_snr && (!snr_db || !counters)) || n_trials < 0) return set_error(OFDM_E_ARG, "bad sweep args");
    if (cfg->channel != OFDM_CHAN_AWGN) return set_error(OFDM_E_ARG, "frame mode models the AWGN channel only");
    if (cfg->noise == OFDM_NOISE_COMPLEX) return set_error(OFDM_E_ARG, "frame mode noise is real (OFDM.c:651) or none");
    if (n_snr == 0) return OFDM_OK;
    HIPOK(hipSetDevice(c->device));
    if ((rc = ensure_wave(c, cfg->conv, cfg->payload))) return rc;
    const size_t cbytes = (size_t)n_snr * OFDM_NCOUNTERS * 8;
    const size_t pbytes = packet_idx ? (size_t)n_snr * n_trials * 4 : 0;
    if ((rc = c->ensure(&c->d_cnt, &c->cap_cnt, cbytes + pbytes + 256))) return rc;
    HIPOK(hipMemsetAsync(c->d_cnt, 0, cbytes, c->stream));
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
        c->tic(Ctx::K_FRAME);
        hipLaunchKernelGGL(frame_rx_kernel, dim3(frame_grid(c, n_trials * a.n_snr)), dim3(64), 0, c->stream, a);
        c->toc();
        HIPOK(hipGetLastError());
    }
    HIPOK(hipMemcpyAsync(counters, c->d_cnt, cbytes, hipMemcpyDeviceToHost, c->stream));
    if (dp) HIPOK(hipMemcpyAsync(packet_idx, dp, pbytes, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    return OFDM_OK;
}

}  // extern "C"
