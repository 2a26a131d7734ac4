// ofdm_symbol.hip -- symbol-mode kernels for gfx950 (MI355X): K1 batched FFT, K2 Tx builder,
// K3 fused AWGN/Rayleigh + receiver chain with counters.  DESIGN.md §2-§4 describe layout,
// roofline and the RNG spec; the per-stage reference lines are cited inline.
//
// Mapping: ONE LANE OWNS ONE 64-SAMPLE WINDOW (a data symbol or one long-training symbol); its
// 64-point FFT lives in that lane's VGPRs (ofdm_device.h).  In LS mode the four lanes of a DPP
// quad carry one frame {LTF1, LTF2, D0, D1}: the LS estimate H = 0.5(F1+F2)conj(Lf)
// (OFDM.c:830-850) is formed with two quad broadcasts, no LDS.
//
// Register discipline: the first radix-4 stage is fused with sample generation (load + channel +
// noise) four butterflies at a time, then the four 16-point sub-FFTs run one after another and
// each sub-block's bins are consumed (demapped or stored) at once.  sched_fence() pins that
// order so the live set stays ~128 VGPRs + temporaries (3 waves/SIMD, no scratch).
#include "ofdm_internal.h"
#include "ofdm_rxcommon.h"

#ifndef OFDM_RX_WAVES_PER_SIMD
#define OFDM_RX_WAVES_PER_SIMD 2
#endif

namespace ofdm {

// ======================================================================== K1: batched FFT
// One wave = 64 transforms.  Coalesced 16-B loads into a padded LDS image (row = 64 float2 + 1
// pad: conflict-free ds_read_b64 per lane-row), each lane then runs its own register FFT.
constexpr int K1_ROW = 65;  // float2 per LDS row

template <bool INV, int CONV>
__global__ __launch_bounds__(64, 2) void fft64_kernel(const float2 *__restrict__ in, float2 *__restrict__ out,
                                                      int64_t n) {
    __shared__ float2 lds[64 * K1_ROW];
    const int lane = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * 64;
    const int64_t nt = (n - base) < 64 ? (n - base) : 64;   // transforms in this wave
    const float4 *src = reinterpret_cast<const float4 *>(in + base * 64);
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
        const int e = k * 128 + lane * 2;   // float2 element index within the wave's block
        const int row = e >> 6, col = e & 63;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nt) v = src[e >> 1];
        lds[row * K1_ROW + col] = make_float2(v.x, v.y);
        lds[row * K1_ROW + col + 1] = make_float2(v.z, v.w);
    }
    __syncthreads();
    float2 x[64];
    const float2 *row = lds + lane * K1_ROW;
    static_for<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        static_for<0, 16>([&](auto pc) {
            constexpr int n = 16 * (decltype(pc)::value >> 2) + 4 * g + (decltype(pc)::value & 3);
            float2 v = row[n];
            // fft(): DFT of x[n](-1)^n = fftshift(DFT(x)) (OFDM.c:314-318);
            // ifft(): X~[i] = X[i](-1)^i for the C convention (D5), none for MATLAB
            if constexpr ((!INV || CONV == OFDM_CONV_C) && (n & 1)) v = make_float2(-v.x, -v.y);
            x[n] = v;
        });
        static_for<0, 4>([&](auto ic) { dif_stage1<INV, 4 * g + decltype(ic)::value>(x); });
        sched_fence();
    });
    __syncthreads();   // every lane has read its row
    float2 *orow = lds + lane * K1_ROW;
    static_for<0, 4>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        dif_sub16<INV, R>(x);
        static_for<0, 16>([&](auto kc) {
            constexpr int k = 4 * decltype(kc)::value + R;     // bins with k & 3 == R
            float2 v = x[digit_rev4(k)];
            if constexpr (INV) v = cscale(v, (k & 1) ? -1.0f / 64.0f : 1.0f / 64.0f);   // (-1)^n / 64
            orow[k] = v;
        });
        sched_fence();
    });
    __syncthreads();
    float4 *dst = reinterpret_cast<float4 *>(out + base * 64);
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
        const int e = k * 128 + lane * 2;
        const int r = e >> 6, col = e & 63;
        if (r < nt) {
            const float2 a = lds[r * K1_ROW + col], b = lds[r * K1_ROW + col + 1];
            dst[e >> 1] = make_float4(a.x, a.y, b.x, b.y);
        }
    }
}

// ======================================================================== K2: Tx builder
// One lane = one data symbol: bits -> QPSK (OFDM.c:415-433) -> subcarrier map + pilots
// (OFDM.c:523-548) -> ifft (OFDM.c:320-339, convention D5) -> CP (OFDM.c:559-565) -> HBM.
template <int CONV>
__global__ __launch_bounds__(256, 3) void tx_symbols_kernel(TxArgs a) {
    const int64_t sidx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // symbol within batch
    if (sidx >= a.n_sym) return;
    const uint64_t s = a.first_symbol + (uint64_t)sidx;
    uint32_t w[3];
    if (a.payload == OFDM_PAYLOAD_RANDOM) {
        const uint4 o = philox10((uint32_t)s, (uint32_t)(s >> 32), 0u, STREAM_BITS, a.k0, a.k1);
        w[0] = o.x; w[1] = o.y; w[2] = o.z;
    } else {
        const int r = (int)(s & 1);
        w[0] = a.table[3 * r]; w[1] = a.table[3 * r + 1]; w[2] = a.table[3 * r + 2];
    }
    float2 X[64];
    static_for<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        uint32_t wg[3] = {w[0], w[1], w[2]};
        opaque(wg[0]); opaque(wg[1]); opaque(wg[2]);
        static_for<0, 16>([&](auto pc) {
            constexpr int i = 16 * (decltype(pc)::value >> 2) + 4 * g + (decltype(pc)::value & 3);
            X[i] = tx_bin<CONV, i>(wg);
        });
        static_for<0, 4>([&](auto ic) { dif_stage1<true, 4 * g + decltype(ic)::value>(X); });
        sched_fence();
    });
    const int64_t tile = sidx >> 5;
    const int slot = (int)(sidx & 31);
    float2 *dst = a.tx + tile * (SYM_SAMPLES * TILE_SYMBOLS) + slot;
    static_for<0, 4>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        dif_sub16<true, R>(X);
        gf2 *d = (gf2 *)dst;
        opaque(d);
        static_for<0, 16>([&](auto nc) {
            constexpr int n = 4 * decltype(nc)::value + R;                   // time samples n & 3 == R
            const float2 v = cscale(X[digit_rev4(n)], (n & 1) ? -1.0f / 64.0f : 1.0f / 64.0f);
            gst(d, (16 + n) * TILE_SYMBOLS, v);
            if constexpr (n >= 48) gst(d, (n - 48) * TILE_SYMBOLS, v);           // CP = last 16 samples
        });
        sched_fence();
    });
    uint32_t *bd = a.bits + tile * (3 * TILE_SYMBOLS) + slot;
    bd[0] = w[0]; bd[TILE_SYMBOLS] = w[1]; bd[2 * TILE_SYMBOLS] = w[2];
}

// ======================================================================== K3: receiver chain
// Clean sample n of a window: data windows read row 16+n of the Tx tile (n >= -3 reaches into the
// CP), LTF windows read the cyclic training symbol T[(n + 64) & 63].
// P is a global (gcf2) or LDS (lcf2) view.
template <typename P>
struct WindowSrc {
    P *p;                // data: &tile[16][slot]; LTF: T
    int stride;          // 32 (data) or 1 (LTF)
    bool circ;           // LTF
};
template <typename P>
__device__ __forceinline__ float2 src_at(P *p, int stride, bool circ, int n) {
    if (n >= 0) return ld2(p, n * stride);
    return circ ? ld2(p, 64 + n) : ld2(p, n * stride);
}

// Load + channel + AWGN for samples n0..n0+3, times (-1)^n (fft() = DFT of x(-1)^n, OFDM.c:314-318).
// Noise sample at frame time t uses Gaussian t (real) or 2t, 2t+1 (complex) of the frame's stream
// (DESIGN.md §3); AWGN is real-only as OFDM.c:651 really does (D7).
template <int NOISE, int CHAN, int N0, typename WS>
__device__ __forceinline__ void rx_block(float2 (&x)[64], const WS &src, uint32_t f_lo, uint32_t f_hi,
                                         uint32_t t0, uint32_t q, float sigma, uint32_t k0, uint32_t k1,
                                         const float2 (&h)[4]) {
    // re-materialise per block: keeps LICM from hoisting 16 blocks' worth of addresses / round-1 products
    auto p = src.p;
    uint32_t flo = f_lo, fhi = f_hi, tb = t0;
    opaque(p); opaque(flo); opaque(fhi); opaque(tb);
    f_lo = flo; f_hi = fhi; t0 = tb;
    float z[8];
    if constexpr (NOISE == OFDM_NOISE_REAL) {
        const Gauss4 g = gauss4(f_lo, f_hi, (t0 >> 2) + (N0 >> 2), STREAM_NOISE | q, k0, k1);
        z[0] = g.z[0]; z[1] = g.z[1]; z[2] = g.z[2]; z[3] = g.z[3];
    } else if constexpr (NOISE == OFDM_NOISE_COMPLEX) {
        const Gauss4 g0 = gauss4(f_lo, f_hi, (t0 >> 1) + (N0 >> 1), STREAM_NOISE | q, k0, k1);
        const Gauss4 g1 = gauss4(f_lo, f_hi, (t0 >> 1) + (N0 >> 1) + 1, STREAM_NOISE | q, k0, k1);
        z[0] = g0.z[0]; z[1] = g0.z[1]; z[2] = g0.z[2]; z[3] = g0.z[3];
        z[4] = g1.z[0]; z[5] = g1.z[1]; z[6] = g1.z[2]; z[7] = g1.z[3];
    }
    float2 c[7];
    if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {
        static_for<0, 7>([&](auto ic) { c[decltype(ic)::value] = src_at(p, src.stride, src.circ, N0 - 3 + decltype(ic)::value); });
    } else {
        static_for<0, 4>([&](auto ic) { c[3 + decltype(ic)::value] = src_at(p, src.stride, src.circ, N0 + decltype(ic)::value); });
    }
    static_for<0, 4>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int n = N0 + i;
        float2 y = c[3 + i];
        if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {   // y[t] = sum_l h_l x[t - l], 4 taps < CP
            y = cadd(cadd(cmul(h[0], c[3 + i]), cmul(h[1], c[2 + i])), cadd(cmul(h[2], c[1 + i]), cmul(h[3], c[i])));
        }
        if constexpr (NOISE == OFDM_NOISE_REAL) {
            y.x = fmaf(sigma, z[i], y.x);
        } else if constexpr (NOISE == OFDM_NOISE_COMPLEX) {
            const float sh = sigma * INV_SQRT2;
            y.x = fmaf(sh, z[2 * i], y.x);
            y.y = fmaf(sh, z[2 * i + 1], y.y);
        }
        if constexpr (n & 1) y = make_float2(-y.x, -y.y);
        x[n] = y;
    });
}

// generate the window fused with the first radix-4 stage (4 butterflies per group)
template <int NOISE, int CHAN, typename WS>
__device__ __forceinline__ void rx_window_stage1(float2 (&x)[64], const WS &src, uint32_t f_lo,
                                                 uint32_t f_hi, uint32_t t0, uint32_t q, float sigma,
                                                 uint32_t k0, uint32_t k1, const float2 (&h)[4]) {
    static_for<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        rx_block<NOISE, CHAN, 4 * g>(x, src, f_lo, f_hi, t0, q, sigma, k0, k1, h);
        rx_block<NOISE, CHAN, 16 + 4 * g>(x, src, f_lo, f_hi, t0, q, sigma, k0, k1, h);
        rx_block<NOISE, CHAN, 32 + 4 * g>(x, src, f_lo, f_hi, t0, q, sigma, k0, k1, h);
        rx_block<NOISE, CHAN, 48 + 4 * g>(x, src, f_lo, f_hi, t0, q, sigma, k0, k1, h);
        static_for<0, 4>([&](auto ic) { dif_stage1<false, 4 * g + decltype(ic)::value>(x); });
        sched_fence();
    });
}

// Shared tail: FFT sub-blocks + demap, per-frame combine of the two data symbols (quad xor-1
// partner), counters.  `leader` lanes (one per valid frame) contribute.
template <bool DUMP, int KIND, typename HF>
__device__ __forceinline__ void finish_symbol(float2 (&x)[64], const uint32_t (&w)[3], HF &&Hof, float2 *dump_eq,
                                              uint32_t *dump_bits, bool leader, unsigned long long *slots) {
    SymState st;
    sym_init(st);
    static_for<0, 4>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        dif_sub16<false, R>(x);
        demap_sub<DUMP, R, KIND>(x, w, Hof, dump_eq, st);
        sched_fence();
    });
    if constexpr (DUMP) {
        if (dump_bits) { dump_bits[0] = st.d[0]; dump_bits[1] = st.d[1]; dump_bits[2] = st.d[2]; }
    }
    const float evm = finish_evm<KIND>(st);
    const float e_other = dpp_f<DPP_QUAD_XOR1>(evm);
    const uint32_t be_other = dpp_u<DPP_QUAD_XOR1>(st.be);
    const uint32_t ax_other = dpp_u<DPP_QUAD_XOR1>(st.ax);
    FrameAcc acc;
    if (leader) frame_metrics(acc, evm + e_other, st.be + be_other, st.ax + ax_other);
    flush_wave(acc, slots);
}

// ---- LS estimate: quad = {LTF1, LTF2, D0, D1} of one frame; wave = 16 frames = one tile ----
// Each wave stages the rows of its tile the windows read (16..79, or 12..79 when the 4-tap channel
// reaches 3 samples into the CP) into its own LDS slice once, with global_load_lds_dwordx4 (1 KB per
// wave instruction), so the n_snr passes over the tile read LDS instead of re-fetching HBM/L2.
template <int CHAN>
struct LsStage {
    static constexpr int R0 = CHAN == OFDM_CHAN_RAYLEIGH4 ? 12 : 16;
    static constexpr int ROWS = SYM_SAMPLES - R0;
    static constexpr int BYTES = ROWS * TILE_SYMBOLS * 8;
    static constexpr int CHUNKS = BYTES / 1024;
    static_assert(BYTES % 1024 == 0, "staged rows must be whole 1 KB wave chunks");
};

template <int NOISE, int CHAN, bool DUMP>
__global__ __launch_bounds__(256, OFDM_RX_WAVES_PER_SIMD) void rx_ls_kernel(RxArgs a) {
    using St = LsStage<CHAN>;
    __shared__ unsigned long long sacc[OFDM_MAX_SNR][8];
    __shared__ __attribute__((aligned(16))) float2 s_tile[4][St::ROWS * TILE_SYMBOLS];
    __shared__ float2 s_ltf[64];
    for (int i = threadIdx.x; i < a.n_snr * 8; i += blockDim.x) (&sacc[0][0])[i] = 0ull;
    if (threadIdx.x < 64) s_ltf[threadIdx.x] = a.ltf[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int role = lane & 3, fi = lane >> 2;
    const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    // window start on the frame timeline: LTF1 192, LTF2 256, D0 336, D1 416
    const uint32_t t0 = role == 0 ? 192u : role == 1 ? 256u : (role == 2 ? 336u : 416u);
    const bool is_data = role >= 2;
    const int slot = 2 * fi + (role & 1);
    float2 *my_tile = s_tile[wv];

    for (int64_t tile = wave_id; tile < a.n_tiles; tile += n_waves) {
        const int64_t fl = tile * TILE_FRAMES + fi;
        const bool valid = fl < a.n_frames;
        const uint64_t f = a.first_frame + (uint64_t)fl;
        const uint32_t f_lo = (uint32_t)f, f_hi = (uint32_t)(f >> 32);
        {
            // previous tile's LDS reads were consumed by its FFTs, so the slice is free to overwrite
            const char *g = (const char *)(a.tx + tile * (SYM_SAMPLES * TILE_SYMBOLS) + St::R0 * TILE_SYMBOLS) + lane * 16;
            static_for<0, St::CHUNKS>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(g + c * 1024),
                                                 (__attribute__((address_space(3))) void *)((char *)my_tile + c * 1024),
                                                 16, 0, 0);
            });
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        WindowSrc<lcf2> src;
        src.p = is_data ? (lcf2 *)(my_tile + (16 - St::R0) * TILE_SYMBOLS + slot) : (lcf2 *)s_ltf;
        src.stride = is_data ? TILE_SYMBOLS : 1;
        src.circ = !is_data;
        uint32_t w[3] = {0u, 0u, 0u};
        if (is_data) {
            const uint32_t *bp = a.bits + tile * (3 * TILE_SYMBOLS) + slot;
            w[0] = bp[0]; w[1] = bp[TILE_SYMBOLS]; w[2] = bp[2 * TILE_SYMBOLS];
        }
        float2 h[4] = {make_float2(1.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
        if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) channel_taps(f_lo, f_hi, a.k0, a.k1, h);

        for (int q = 0; q < a.n_snr; ++q) {
            WindowSrc<lcf2> s = src;
            uint32_t wq[3] = {w[0], w[1], w[2]};
            uint32_t flo = f_lo, fhi = f_hi;
            float2 hq[4] = {h[0], h[1], h[2], h[3]};
            opaque(s.p); opaque(wq[0]); opaque(wq[1]); opaque(wq[2]); opaque(flo); opaque(fhi);
            if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {
                static_for<0, 4>([&](auto lc) { opaque(hq[decltype(lc)::value].x); opaque(hq[decltype(lc)::value].y); });
            }
            float2 x[64];
            rx_window_stage1<NOISE, CHAN>(x, s, flo, fhi, t0, (uint32_t)(a.q_base + q), a.sigma[q], a.k0, a.k1, hq);
            float2 *dump_eq = nullptr;
            uint32_t *dump_bits = nullptr;
            if constexpr (DUMP) {
                if (is_data && valid) {
                    const int64_t r = ((int64_t)q * a.dump_frames + fl) * 2 + (role & 1);
                    dump_eq = a.dump_eq + r * 48;
                    dump_bits = a.dump_bits + r * 3;
                }
            }
            // H[k] = 0.5 (F1[k] + F2[k]) conj(Lf[k]), Lf = +-1 on data bins (OFDM.c:846-849)
            auto Hof = [&](float2 Y, auto binc) { return ls_equalise<decltype(binc)::value>(Y); };
            finish_symbol<DUMP, 2>(x, wq, Hof, dump_eq, dump_bits, role == 2 && valid, sacc[q]);
        }
    }
    block_flush(a, sacc);
}

// ---- ideal channel knowledge: every lane a data symbol; wave = 2 tiles = 32 frames ----
template <int CONV, int NOISE, int CHAN, bool DUMP>
__global__ __launch_bounds__(256, OFDM_RX_WAVES_PER_SIMD) void rx_ideal_kernel(RxArgs a) {
    __shared__ unsigned long long sacc[OFDM_MAX_SNR][8];
    for (int i = threadIdx.x; i < a.n_snr * 8; i += blockDim.x) (&sacc[0][0])[i] = 0ull;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int d = lane & 1;
    const uint32_t t0 = 336u + 80u * (uint32_t)d;
    const int64_t n_pairs = (a.n_tiles + 1) >> 1;
    for (int64_t pr = wave_id; pr < n_pairs; pr += n_waves) {
        const int64_t tile = 2 * pr + (lane >> 5);
        const int slot = lane & 31;
        const int64_t fl = tile * TILE_FRAMES + (slot >> 1);
        const bool valid = fl < a.n_frames;
        const uint64_t f = a.first_frame + (uint64_t)fl;
        const uint32_t f_lo = (uint32_t)f, f_hi = (uint32_t)(f >> 32);
        WindowSrc<gcf2> src;
        src.p = (gcf2 *)(a.tx + tile * (SYM_SAMPLES * TILE_SYMBOLS) + 16 * TILE_SYMBOLS + slot);
        src.stride = TILE_SYMBOLS;
        src.circ = false;
        const uint32_t *bp = a.bits + tile * (3 * TILE_SYMBOLS) + slot;
        uint32_t w[3] = {bp[0], bp[TILE_SYMBOLS], bp[2 * TILE_SYMBOLS]};
        float2 h[4] = {make_float2(1.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
        if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) channel_taps(f_lo, f_hi, a.k0, a.k1, h);
        for (int q = 0; q < a.n_snr; ++q) {
            WindowSrc<gcf2> s = src;
            uint32_t wq[3] = {w[0], w[1], w[2]};
            uint32_t flo = f_lo, fhi = f_hi;
            float2 hq[4] = {h[0], h[1], h[2], h[3]};
            opaque(s.p); opaque(wq[0]); opaque(wq[1]); opaque(wq[2]); opaque(flo); opaque(fhi);
            if constexpr (CHAN == OFDM_CHAN_RAYLEIGH4) {
                static_for<0, 4>([&](auto lc) { opaque(hq[decltype(lc)::value].x); opaque(hq[decltype(lc)::value].y); });
            }
            float2 x[64];
            rx_window_stage1<NOISE, CHAN>(x, s, flo, fhi, t0, (uint32_t)(a.q_base + q), a.sigma[q], a.k0, a.k1, hq);
            float2 *dump_eq = nullptr;
            uint32_t *dump_bits = nullptr;
            if constexpr (DUMP) {
                if (valid) {
                    const int64_t r = ((int64_t)q * a.dump_frames + fl) * 2 + d;
                    dump_eq = a.dump_eq + r * 48;
                    dump_bits = a.dump_bits + r * 3;
                }
            }
            // perfect CSI: H[i] = c_i sum_l h_l e^{-j2pi(i-32)l/64}, c_i = (-1)^i for the C ifft (D5)
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
            finish_symbol<DUMP, KIND>(x, wq, Hof, dump_eq, dump_bits, d == 0 && valid, sacc[q]);
        }
    }
    block_flush(a, sacc);
}

// ======================================================================== launchers
template <bool INV>
static void launch_fft_conv(int conv, dim3 g, hipStream_t st, const float2 *in, float2 *out, int64_t n) {
    if (conv == OFDM_CONV_C) hipLaunchKernelGGL((fft64_kernel<INV, OFDM_CONV_C>), g, dim3(64), 0, st, in, out, n);
    else hipLaunchKernelGGL((fft64_kernel<INV, OFDM_CONV_MATLAB>), g, dim3(64), 0, st, in, out, n);
}

void launch_fft64(hipStream_t st, const float2 *in, float2 *out, int64_t n, int inverse, int conv) {
    const dim3 g((unsigned)((n + 63) / 64));
    if (inverse) launch_fft_conv<true>(conv, g, st, in, out, n);
    else launch_fft_conv<false>(OFDM_CONV_C, g, st, in, out, n);
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

int rx_grid(const ofdm_cfg &cfg, int64_t n_tiles, int device) {
    // waves needed: one per tile (LS) or per tile pair (ideal); 4 waves per block
    const int64_t waves = cfg.est == OFDM_EST_LS ? n_tiles : (n_tiles + 1) / 2;
    const int64_t need = (waves + 3) / 4;
    int per_cu = 0, cus = 0;
    const void *k = cfg.est == OFDM_EST_LS
        ? reinterpret_cast<const void *>(&rx_ls_kernel<OFDM_NOISE_REAL, OFDM_CHAN_AWGN, false>)
        : reinterpret_cast<const void *>(&rx_ideal_kernel<OFDM_CONV_C, OFDM_NOISE_REAL, OFDM_CHAN_AWGN, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess || per_cu < 1) per_cu = 2;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
    const int64_t cap = (int64_t)per_cu * cus;
    const int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace ofdm
