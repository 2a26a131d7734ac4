// ofdm_rxcommon.h -- receiver helpers shared by the symbol-mode (K3) and frame-mode (K4)
// kernels: DPP quad exchanges, per-symbol demap + metrics, per-frame counters.
#pragma once
#include "ofdm_internal.h"

namespace ofdm {

// Tx subcarrier value of fftshifted bin BIN for a symbol whose payload bits are w (MSB first):
// QPSK data (OFDM.c:415-433), pilots {1,1,1,-1} (OFDM.c:523-544), nulls/DC 0; times (-1)^BIN for
// the C ifft convention (D5).
template <int CONV, int BIN>
__device__ __forceinline__ float2 tx_bin(const uint32_t (&w)[3]) {
    constexpr float sgn = (CONV == OFDM_CONV_C && (BIN & 1)) ? -1.0f : 1.0f;   // ifftshift+fftshift (D5)
    constexpr int m = data_index(BIN);
    if constexpr (m >= 0) {
        const uint32_t b0 = bit_of(w, 2 * m), b1 = bit_of(w, 2 * m + 1);
        // 00:(+,+) 01:(-,+) 10:(-,-) 11:(+,-): re > 0 iff b0 == b1, im > 0 iff b0 == 0 (D10)
        const float re = (b0 == b1) ? sgn * INV_SQRT2 : -sgn * INV_SQRT2;
        const float im = b0 ? -sgn * INV_SQRT2 : sgn * INV_SQRT2;
        return make_float2(re, im);
    } else {
        return make_float2(sgn * pilot_at(BIN), 0.0f);    // pilots {1,1,1,-1}; nulls and DC 0
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ float2 dpp_c(float2 v) { return make_float2(dpp_f<CTRL>(v.x), dpp_f<CTRL>(v.y)); }
constexpr int DPP_QUAD_BCAST0 = 0x00;   // quad_perm [0,0,0,0]

__device__ __forceinline__ void channel_taps(uint32_t f_lo, uint32_t f_hi, uint32_t k0, uint32_t k1, float2 (&h)[4]) {
    const Gauss4 a = gauss4(f_lo, f_hi, 0u, STREAM_CHAN, k0, k1);
    const Gauss4 b = gauss4(f_lo, f_hi, 1u, STREAM_CHAN, k0, k1);
    const float s = 0.35355339059327376220f;   // sqrt(1/8): CN(0, 1/4) per tap
    h[0] = make_float2(s * a.z[0], s * a.z[1]);
    h[1] = make_float2(s * a.z[2], s * a.z[3]);
    h[2] = make_float2(s * b.z[0], s * b.z[1]);
    h[3] = make_float2(s * b.z[2], s * b.z[3]);
}

// Truth bits in demap order.  The receivers consume the data bins one FFT sub-block at a time: sub-block
// R holds the bins k = 4 kc + R (kc ascending), 12 / 11 / 14 / 11 data bins for R = 0..3.  Demap word
// R of a symbol lists, MSB first, for each of those bins the expected sign of the imaginary axis (b0)
// then of the real axis (b0 ^ b1) -- the non-Gray map of D10: im < 0 iff b0, re < 0 iff b0 != b1 --
// so the receiver walks it with v_add (t + t, a fast-class shift) instead of per-bin shifts.
template <int R>
__host__ __device__ constexpr int demap_bins() {
    int n = 0;
    for (int kc = 0; kc < 16; ++kc) n += data_index(4 * kc + R) >= 0;
    return n;
}
template <int R>
__host__ __device__ inline uint32_t demap_word(const uint32_t w[3]) {
    uint32_t t = 0u;
    int pos = 31;
    for (int kc = 0; kc < 16; ++kc) {
        const int m = data_index(4 * kc + R);
        if (m < 0) continue;
        const uint32_t b0 = (w[(2 * m) >> 5] >> (31 - ((2 * m) & 31))) & 1u;
        const uint32_t b1 = (w[(2 * m + 1) >> 5] >> (31 - ((2 * m + 1) & 31))) & 1u;
        t |= b0 << pos;
        t |= (b0 ^ b1) << (pos - 1);
        pos -= 2;
    }
    return t;
}
__host__ __device__ inline void demap_words(const uint32_t w[3], uint32_t t[4]) {
    t[0] = demap_word<0>(w); t[1] = demap_word<1>(w); t[2] = demap_word<2>(w); t[3] = demap_word<3>(w);
}

// Hermitian bin pairs of the packed real-noise receivers (ofdm_rxpack.hip).  The 48 data bins form 24
// pairs (k, 64 - k), k < 32, listed in the order the receiver consumes them: the pairs of FFT sub-block
// 0 (k = 0 mod 4), of sub-block 2 (k = 2 mod 4), then the odd k (sub-blocks 1 and 3 together).
constexpr int PACK_PAIRS = 24;
__host__ __device__ constexpr int pair_bin(int p) {
    constexpr int8_t K[PACK_PAIRS] = {8, 12, 16, 20, 24, 28, 6, 10, 14, 18, 22, 26, 30,
                                      7, 9, 13, 15, 17, 19, 21, 23, 27, 29, 31};
    return K[p];
}
// Pair-order truth words of one symbol (Tx rows 7..9): for each pair p, bins k then 64 - k, each as
// (b0, b0 ^ b1) MSB first -- 4 bits per pair, 8 pairs per word (the demap_word signs, D10).
__host__ __device__ inline void pair_words(const uint32_t w[3], uint32_t t[3]) {
    t[0] = t[1] = t[2] = 0u;
    for (int p = 0; p < PACK_PAIRS; ++p)
        for (int h = 0; h < 2; ++h) {
            const int bin = h ? 64 - pair_bin(p) : pair_bin(p);
            const int m = data_index(bin);
            const uint32_t b0 = (w[(2 * m) >> 5] >> (31 - ((2 * m) & 31))) & 1u;
            const uint32_t b1 = (w[(2 * m + 1) >> 5] >> (31 - ((2 * m + 1) & 31))) & 1u;
            const int pos = 31 - 4 * (p & 7) - 2 * h;
            t[p >> 3] |= (b0 << pos) | ((b0 ^ b1) << (pos - 1));
        }
}

// Per-symbol decisions + metrics, consumed one FFT sub-block at a time.
//   Z = Y / H (OFDM.c:1044-1052), slicer (OFDM.c:852-871), demap (OFDM.c:873-908), bit compare
//   (OFDM.c:1154-1161), EVM pre/post (OFDM.c:1104-1150).
//
// The equaliser hands back Z = u * g with g > 0, so the slicer decision is the sign of u:
//   KIND 0: g = 1 (ideal AWGN), KIND 1: g = r (ideal ZF, r = 1/|H|^2),
//   KIND 2: g = 2 r (LTF LS: Y / (0.5 Lf S) = 2 Lf Y conj(S) / |S|^2, r = 1/|S|^2).
// With the truth symbol d = (sr c, si c), c = 1/sqrt2, flipping u's sign bits by the demap word's
// expected signs gives u' with
//   |Z - d|^2 = (u'.x g - c)^2 + (u'.y g - c)^2     and     axis error <=> sign bit of u' set,
// so each bin costs two v_add to advance the demap word, one v_bitop3 per axis for the truth (the
// sign mask in a VGPR: an SGPR operand issues at the slow rate), one fma per axis for the EVM and one
// alignbit per axis to collect the errors (popcounted once per sub-block).  Decisions agree with
// "Z > 0" (OFDM.c:858-866) except for an exactly-zero equalised value.
template <int KIND>
struct EqOut {
    float2 u;
    float r;    // unused for KIND 0
};
struct SymState {
    float evm_pre;     // KIND 2: sum of (|Z - d| / 2)^2; scaled once per symbol by finish_evm
    uint32_t be, ax;   // bit errors, slicer axis errors
    uint32_t d[3];     // decided bits, DUMP only
};

__device__ __forceinline__ void sym_init(SymState &st) {
    st.evm_pre = 0.f; st.be = 0u; st.ax = 0u; st.d[0] = st.d[1] = st.d[2] = 0u;
}
template <int KIND>
__device__ __forceinline__ float finish_evm(const SymState &st) { return KIND == 2 ? 4.0f * st.evm_pre : st.evm_pre; }

// t + t as a v_add_u32 (fast class): LLVM would otherwise fold it into a v_lshlrev (slow class)
__device__ __forceinline__ uint32_t dbl_u32(uint32_t t) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(t));
    return r;
}

// t: demap word R of this lane's symbol (0 on lanes without a data symbol)
template <bool DUMP, int R, int KIND, typename HF>
__device__ __forceinline__ void demap_sub(const float2 (&x)[64], uint32_t t, HF &&Hof, float2 *dump_eq, SymState &st) {
    uint32_t sm;
    asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(sm));
    constexpr float cd = KIND == 2 ? 0.5f * INV_SQRT2 : INV_SQRT2;
    uint32_t em = 0u;     // per bin: re error then im error, shifted in from bit 0
    static_for<0, 16>([&](auto kc) {
        constexpr int bin = 4 * decltype(kc)::value + R;
        constexpr int m = data_index(bin);
        if constexpr (m >= 0) {
            const EqOut<KIND> e = Hof(x[digit_rev4(bin)], std::integral_constant<int, bin>{});
            const uint32_t ti = t, tr = dbl_u32(t);
            t = dbl_u32(tr);
            // u' = u ^ (t & 0x80000000): bitop3 table a ^ (b & c) = 0x78
            const uint32_t ur = __builtin_amdgcn_bitop3_b32(__float_as_uint(e.u.x), tr, sm, 0x78);
            const uint32_t ui = __builtin_amdgcn_bitop3_b32(__float_as_uint(e.u.y), ti, sm, 0x78);
            float ex, ey;
            if constexpr (KIND == 0) {
                ex = __uint_as_float(ur) - cd;
                ey = __uint_as_float(ui) - cd;
            } else {
                ex = fmaf(__uint_as_float(ur), e.r, -cd);
                ey = fmaf(__uint_as_float(ui), e.r, -cd);
            }
            st.evm_pre = fmaf(ex, ex, fmaf(ey, ey, st.evm_pre));
            em = __builtin_amdgcn_alignbit(em, ur, 31);
            em = __builtin_amdgcn_alignbit(em, ui, 31);
            if constexpr (DUMP) {
                const float g = KIND == 0 ? 1.0f : KIND == 1 ? e.r : 2.0f * e.r;
                const float2 z = KIND == 0 ? e.u : make_float2(e.u.x * g, e.u.y * g);
                if (dump_eq) dump_eq[m] = z;
                const uint32_t pr = z.x > 0.f, pi = z.y > 0.f;
                constexpr int wi = (2 * m) >> 5;
                constexpr int s0 = 31 - ((2 * m) & 31), s1 = 31 - ((2 * m + 1) & 31);
                st.d[wi] |= ((pi ^ 1u) << s0) | ((pr ^ pi) << s1);
            }
        }
    });
    // pin the sub-block's EVM terms here: left alone, LLVM sinks the fma chain to its single use after
    // the last sub-block and keeps every bin's u' alive until then (the spills of round 1)
    opaque(st.evm_pre);
    // im errors at even positions, re errors at odd: b0 wrong <=> im wrong, b1 wrong <=> re ^ im
    st.ax += __popc(em);
    st.be += __popc(em & 0x55555555u) + __popc((em ^ (em >> 1)) & 0x55555555u);
}

// LTF least-squares equaliser for a quad {LTF1 + LTF2, -, D0, D1} of one frame (frame_sym_kernel): the LTF pair
// arrives as one window, so lane 0's spectrum is S = FFT(LTF1 + LTF2) = F1 + F2 (fft() is linear), H = 0.5 Lf S
// (OFDM.c:846-849), Z = Y / H = 2 Lf Y conj(S) / |S|^2 (OFDM.c:1044-1052).
template <int BIN>
__device__ __forceinline__ EqOut<2> ls_equalise(float2 Y) {
    const float2 S = dpp_c<DPP_QUAD_BCAST0>(Y);
    EqOut<2> e;
    e.r = __builtin_amdgcn_rcpf(fmaf(S.x, S.x, S.y * S.y));
    e.u = cscale(cmulc(Y, S), (float)ltf_sign(BIN));
    return e;
}

// Equaliser objects for finish_symbol: operator()(Y, bin) -> EqOut, and prefetch<R>(x) called once
// per FFT sub-block before its bins are consumed (LDS-crossbar fetches issued as one batch).
template <typename F>
struct EqFn {
    F f;
    template <int R>
    __device__ __forceinline__ void prefetch(const float2 (&)[64]) {}
    template <typename B>
    __device__ __forceinline__ auto operator()(float2 Y, B b) { return f(Y, b); }
};
template <typename F>
__device__ __forceinline__ EqFn<F> eq_fn(F f) { return EqFn<F>{f}; }

// Frame-level counters of one frame's leader lane.  They go straight into the block's LDS slots,
// one ds_add_u64 per lane and slot (the LDS pipe serialises the lanes; no VALU wave reduction).
// Slots of sacc[q]:
//   0: bit errors | slicer axis errors << 32      1: frame errors | finite post-slicer EVM_dB << 32
//   2: EVM_PRE_Q      3: EVMDB_PRE_Q      4: EVMDB_POST_Q
// A 32-bit field cannot carry into its neighbour: one launch covers at most MAX_BATCH_FRAMES = 2^23
// frames, and 2^23 x 192 < 2^32.
struct FrameAcc {
    uint64_t errs = 0, frames = 0;     // packed slots 0 and 1
    int64_t pre_q = 0, dbpre_q = 0, dbpost_q = 0;
};

// x 2^20 rounded to nearest even, as the oracle's q20(): x >= 0 (a frame's sum |z - d|^2)
__device__ __forceinline__ int64_t q20_nonneg(float x) {
    const float v = __builtin_rintf(x * (float)OFDM_EVM_Q_SCALE);      // integer-valued
    const float hi = __builtin_floorf(v * 0x1p-32f);
    const uint32_t lo = (uint32_t)fmaf(hi, -0x1p32f, v);                 // exact: 0 <= v - hi 2^32 < 2^32
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | lo);
}
// |x| 2^20 < 2^31: a frame's EVM_dB (floor -400 dB; 10 log10(FLT_MAX / 96) < 366 dB)
__device__ __forceinline__ int64_t q20_db(float db) {
    return (int64_t)(int32_t)__builtin_rintf(db * (float)OFDM_EVM_Q_SCALE);
}

__device__ __forceinline__ void frame_metrics(FrameAcc &acc, float fe_pre, uint32_t ferr, uint32_t fax) {
    // per-frame EVM_dB = 10 log10(sum|e|^2 / N), N = 96 terms (48 subcarriers x D = 2, OFDM.c:1124-1126),
    // as 10 log10(2) (log2(sum) - log2 96); floor -400 dB.  After the slicer sum|s - d|^2 = 2 fax
    // (OFDM.c:1128-1150): 10 log10(2 fax / 96).
    constexpr float K = 3.01029995663981195214f, L96 = 6.58496250072115618146f;
    acc.errs = (uint64_t)ferr | ((uint64_t)fax << 32);
    acc.frames = (uint64_t)(ferr > 0u) | ((uint64_t)(fax > 0u) << 32);
    acc.pre_q = q20_nonneg(fe_pre);
    const float lg = K * (__builtin_amdgcn_logf(fe_pre) - L96);
    acc.dbpre_q = q20_db(fe_pre > 0.f ? fmaxf(lg, -400.0f) : -400.0f);
    acc.dbpost_q = fax > 0u ? q20_db(K * (__builtin_amdgcn_logf((float)fax) + (1.0f - L96))) : 0;
}

__device__ __forceinline__ void flush_lanes(const FrameAcc &acc, bool leader, unsigned long long *slots /*[8]*/) {
    if (leader) {
        atomicAdd(&slots[0], (unsigned long long)acc.errs);
        atomicAdd(&slots[1], (unsigned long long)acc.frames);
        atomicAdd(&slots[2], (unsigned long long)acc.pre_q);
        atomicAdd(&slots[3], (unsigned long long)acc.dbpre_q);
        atomicAdd(&slots[4], (unsigned long long)acc.dbpost_q);
    }
}

// term k of an SNR point's LDS slots -> (counter index, value)
__device__ __forceinline__ int slot_term(const unsigned long long *s, int k, unsigned long long &v) {
    switch (k) {
        case 0: v = s[0] & 0xffffffffull; return OFDM_C_BIT_ERR;
        case 1: v = s[0] >> 32; return OFDM_C_EVM_POST_AXIS;
        case 2: v = s[1] & 0xffffffffull; return OFDM_C_FRAME_ERR;
        case 3: v = s[1] >> 32; return OFDM_C_EVMDB_POST_FINITE;
        case 4: v = s[2]; return OFDM_C_EVM_PRE_Q;
        case 5: v = s[3]; return OFDM_C_EVMDB_PRE_Q;
        default: v = s[4]; return OFDM_C_EVMDB_POST_Q;
    }
}

template <int S>   // slots per SNR point in the block's LDS accumulators (>= 5); tid = threadIdx.x
__device__ __forceinline__ void block_flush(const RxArgs &a, unsigned long long (*sacc)[S], int tid) {
    __syncthreads();
    for (int i = tid; i < a.n_snr * 7; i += blockDim.x) {
        const int q = i / 7, k = i % 7;
        unsigned long long v;
        const int ci = slot_term(sacc[q], k, v);
        if (v) atomicAdd(&a.counters[q * OFDM_NCOUNTERS + ci], v);
    }
    if (blockIdx.x == 0) {
        for (int q = tid; q < a.n_snr; q += blockDim.x) {
            unsigned long long *c = a.counters + q * OFDM_NCOUNTERS;
            atomicAdd(&c[OFDM_C_FRAMES], (unsigned long long)a.n_frames);
            atomicAdd(&c[OFDM_C_SYMBOLS], (unsigned long long)(2 * a.n_frames));
            atomicAdd(&c[OFDM_C_BITS], (unsigned long long)(192 * a.n_frames));
            atomicAdd(&c[OFDM_C_EVM_TERMS], (unsigned long long)(96 * a.n_frames));
        }
    }
}
template <int S>
__device__ __forceinline__ void block_flush(const RxArgs &a, unsigned long long (*sacc)[S]) {
    block_flush(a, sacc, (int)threadIdx.x);
}



// K2's work for one data symbol `sidx` of a Tx batch (the Tx kernel, and the packed receiver's group prologue
// when it builds the next chunk's batch): bits -> QPSK (OFDM.c:415-433) -> subcarrier map + pilots
// (OFDM.c:523-548) -> ifft (OFDM.c:320-339, convention D5) -> CP (OFDM.c:559-565) -> HBM.
// (TA: TxArgs, or a kernarg-segment view of one: the receiver reads its nested TxArgs through an opaque
// kernarg pointer so that its words are loaded where used, not held in SGPRs across the item loop)
template <int CONV, typename TA>
__device__ __forceinline__ void tx_symbol(const TA &a, int64_t sidx) {
    const uint64_t s = a.first_symbol + (uint64_t)sidx;
    uint32_t w[3];
    if (a.payload == OFDM_PAYLOAD_RANDOM) {
        const uint4 o = philox10((uint32_t)s, (uint32_t)(s >> 32), 0u, STREAM_BITS, a.k0, a.k1);
        w[0] = o.x; w[1] = o.y; w[2] = o.z;
    } else {
        const int r = (int)(s % (uint64_t)a.table_frames);
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
    // row-major batch: sample n of symbol sidx at tx[n * pitch + sidx]; the row base
    // is wave-uniform, so each store is saddr + one per-lane offset
    const uint32_t so = (uint32_t)sidx;
    [[maybe_unused]] const int64_t P = a.pitch;
    static_for<0, 4>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        dif_sub16<true, R>(X);
        static_for<0, 16>([&](auto nc) {
            constexpr int n = 4 * decltype(nc)::value + R;                   // time samples n & 3 == R
            const float2 v = cscale(X[digit_rev4(n)], (n & 1) ? -1.0f / 64.0f : 1.0f / 64.0f);
            gst((gf2 *)(a.tx + (16 + n) * P), so, v);
            if constexpr (n >= 48) gst((gf2 *)(a.tx + (n - 48) * P), so, v);   // CP = last 16 samples
        });
        sched_fence();
    });
    a.bits[so] = w[0];
    a.bits[P + so] = w[1];
    a.bits[2 * P + so] = w[2];
    // rows 3..6: the receivers' demap words (ofdm_rxcommon.h)
    a.bits[3 * P + so] = demap_word<0>(w);
    a.bits[4 * P + so] = demap_word<1>(w);
    a.bits[5 * P + so] = demap_word<2>(w);
    a.bits[6 * P + so] = demap_word<3>(w);
    // rows 7..9: the packed real-noise receivers' pair-order words (ofdm_rxcommon.h pair_words)
    uint32_t pw[3];
    pair_words(w, pw);
    a.bits[7 * P + so] = pw[0];
    a.bits[8 * P + so] = pw[1];
    a.bits[9 * P + so] = pw[2];
}

}  // namespace ofdm
