// ofdm_rxpack.hip -- K3c: the real-noise symbol-mode receivers (configs c2 / c3 / c4, the benchmark, and
// the LS receiver of c5's 4-tap Rayleigh channel, whose taps act on the clean spectra once per group).
//
// The AWGN the reference adds is real-only (OFDM.c:651, D7) and the receiver's fft() is linear
// (OFDM.c:314-318), so the spectrum of a received window is the clean symbol's spectrum plus the
// spectrum of a REAL noise vector:
//   * the clean spectra depend on the frame, not on the SNR point: a group prologue transforms the
//     staged Tx samples of 64 frames once (64-point register FFT per symbol) into LDS;
//   * per SNR point each lane owns ONE frame: its two data windows' noise goes through one complex
//     64-point FFT as d0 + j d1 (Hermitian split per bin pair (k, 64 - k)), and the LTF pair noise
//     n1 + n2 through a 32-point FFT of its even/odd samples packed as e[2m] + j e[2m+1];
//   * the LS estimate S = F1 + F2 = FFT(2T) + FFT(n1 + n2) (OFDM.c:830-850), the ZF equaliser
//     Z = Y / (0.5 Lf S) (OFDM.c:1044-1052) and the slicer/demap/EVM of both data symbols
//     (OFDM.c:852-908, 1104-1161) run in the lane that holds S, bin pair by bin pair.
// Per frame and SNR point that is 1.5 complex FFTs instead of 3, two demaps instead of three
// (the LTF lane of the {E, D0, D1} layout no longer demaps), no clean-sample loads and no
// cross-lane traffic.  The noise draws are the same Philox/Box-Muller values as every other receiver
// (same counters): results agree with the oracle's time-domain chain to fp32 rounding.
#include "ofdm_internal.h"
#include "ofdm_rxcommon.h"

#define OFDM_RX_PACK_WAVES 2          // waves per SIMD the LS receiver is register-budgeted for
#define OFDM_RX_PACK_IDEAL_WAVES 3    // the ideal-CSI receiver (no LTF spectrum) fits 168 VGPRs / 53 KB LDS

namespace ofdm {

constexpr int PK_FRAMES = 64;              // frames per group: one per lane
constexpr int PK_SYMS = 2 * PK_FRAMES;     // data symbols per group

// LDS views (address space 3: keeps ds_read after opaque(), which erases provenance)
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lcf4;
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u2v lcu2;
typedef __attribute__((address_space(3))) f2v lf2;

// LS AWGN receiver: bin-pair LDS operands loaded this many pairs ahead (A/B, profiles/r03/ab_i: c3 +1.2 % at 2,
// +0.6 % at 1; the Rayleigh receiver, whose E spectrum is per frame, gains nothing and keeps 0)
constexpr int PACK_PF = 2;
// the data windows' noise generation: a scheduling fence after every PACK_GEN_SPLIT Philox quarters
constexpr int PACK_GEN_SPLIT = 2;
// the bin-pair loop: a scheduling fence after every PACK_FENCE_PAIRS pairs (keeps the PF loads where written)
constexpr int PACK_FENCE_PAIRS = 2;

// 16-point digit reversal (dif4<16> output order): bin m of a 16-point sub-transform at position rev16(m)
__host__ __device__ constexpr int rev16(int m) { return ((m & 3) << 2) | (m >> 2); }
// position of bin k (0..31) of the 32-point transform (radix-2 stage, then two 16-point dif4)
__host__ __device__ constexpr int pos32(int k) { return (k & 1) ? 16 + rev16(k >> 1) : rev16(k >> 1); }

// The 4-tap channel y[n] = sum_l h_l x[n - l] at FFT bin k of the (-1)^n-modulated window: the taps
// reach 3 samples back, inside the 16-sample cyclic prefix, so over the receiver's window the convolution
// is circular and FFT((-1)^n y[n])[k] = H'[k] FFT((-1)^n x[n])[k] with
// H'[k] = sum_l (-1)^l h_l W64^{kl} (the same frequency response rx_ideal_kernel's ZF uses).
template <int K>
__device__ __forceinline__ float2 chan_bin(const float2 (&h)[4]) {
    float2 H = h[0];
    H = csub(H, twiddle<K * 1, false>(h[1]));
    H = cadd(H, twiddle<K * 2, false>(h[2]));
    return csub(H, twiddle<K * 3, false>(h[3]));
}

// Rayleigh prologue, waves 2-3 (idle while waves 0-1 run the clean FFTs): the channel response of one frame
// at the 12 bin pairs of half HALF, (H'[k], H'[64 - k]) into col[p * PK_FRAMES] (&fce[0][frame]).
template <int HALF>
__device__ __forceinline__ void chan_pairs(const float2 (&h)[4], float4 *col) {
    static_for<12 * HALF, 12 * HALF + 12>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        constexpr int k = pair_bin(p);
        const float2 Hk = chan_bin<k>(h), Hm = chan_bin<64 - k>(h);
        col[p * PK_FRAMES] = make_float4(Hk.x, Hk.y, Hm.x, Hm.y);
        sched_fence();
    });
}

// Group prologue: clean spectrum of symbol `s` (window rows 16..79 of the Tx batch, times (-1)^n for
// fft(), OFDM.c:314-318) -> the 24 bin pairs (C[k], C[64 - k]) of spec[p][half][frame].
__device__ __forceinline__ void clean_spectrum(const RxArgs &a, int64_t s, float4 *spec_col /* &spec[0][half][f] */) {
    gcf2 *src = (gcf2 *)(a.tx + 16 * a.pitch + s);
    int P = (int)a.pitch;
    opaque(P);
    float2 x[64];
    static_for<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        gcf2 *sp = src;
        opaque(sp);
        static_for<0, 16>([&](auto pc) {
            constexpr int n = 16 * (decltype(pc)::value >> 2) + 4 * g + (decltype(pc)::value & 3);
            const float2 v = gld(sp, n * P);
            x[n] = (n & 1) ? make_float2(-v.x, -v.y) : v;
        });
        static_for<0, 4>([&](auto ic) { dif_stage1<false, 4 * g + decltype(ic)::value>(x); });
        sched_fence();
    });
    auto store = [&](auto pc) {
        constexpr int p = decltype(pc)::value;
        constexpr int k = pair_bin(p);
        const float2 c0 = x[digit_rev4(k)], c1 = x[digit_rev4(64 - k)];
        spec_col[p * 2 * PK_FRAMES] = make_float4(c0.x, c0.y, c1.x, c1.y);
    };
    static_for<0, 4>([&](auto rc) { dif_sub16<false, decltype(rc)::value>(x); });
    static_for<0, PACK_PAIRS>(store);
}

// Per-bin demap of one data symbol at one bin: u = Z / g with g > 0 (KIND 0: g = 1, KIND 2: g = 2r),
// the truth signs walked out of t (2 bits, im then re), EVM and slicer errors (demap_sub's arithmetic,
// ofdm_rxcommon.h).  DUMP: the equalised value and the decided bits of data subcarrier m.
template <int KIND, bool DUMP>
__device__ __forceinline__ void demap_bin(float2 u, float r, uint32_t &t, uint32_t sm, float &evm, uint32_t &em,
                                          int m, float2 *dump_eq, uint32_t (&dbits)[3]) {
    constexpr float cd = KIND == 2 ? 0.5f * INV_SQRT2 : INV_SQRT2;
    const uint32_t ti = t, tr = dbl_u32(t);
    t = dbl_u32(tr);
    const uint32_t ur = __builtin_amdgcn_bitop3_b32(__float_as_uint(u.x), tr, sm, 0x78);
    const uint32_t ui = __builtin_amdgcn_bitop3_b32(__float_as_uint(u.y), ti, sm, 0x78);
    float ex, ey;
    if constexpr (KIND == 0) {
        ex = __uint_as_float(ur) - cd;
        ey = __uint_as_float(ui) - cd;
    } else {
        ex = fmaf(__uint_as_float(ur), r, -cd);
        ey = fmaf(__uint_as_float(ui), r, -cd);
    }
    evm = fmaf(ex, ex, fmaf(ey, ey, evm));
    em = __builtin_amdgcn_alignbit(em, ur, 31);
    em = __builtin_amdgcn_alignbit(em, ui, 31);
    if constexpr (DUMP) {
        const float g = KIND == 0 ? 1.0f : 2.0f * r;
        const float2 z = make_float2(u.x * g, u.y * g);
        if (dump_eq) dump_eq[m] = z;
        const uint32_t pr = z.x > 0.f, pi = z.y > 0.f;
        const int wi = (2 * m) >> 5, s0 = 31 - ((2 * m) & 31), s1 = 31 - ((2 * m + 1) & 31);
        dbits[wi] |= ((pi ^ 1u) << s0) | ((pr ^ pi) << s1);
    }
}

// (The ablation builds that priced each stage, OFDM_ABL_* -- tools/stage_mix.py's per-stage budget of the SNR loop
// -- are in git history: profiles/r06/README.md.)
template <typename KS>
__device__ __forceinline__ Noise4 pack_noise(const PhiloxHead &hd, uint32_t c2, const KS &keys, uint32_t k1, float K) {
    uint4 o;
    if constexpr (std::is_same_v<KS, PhiloxKeysV>) o = philox10_c2(hd, c2, keys);
    else o = philox10_c2(hd, c2, keys, k1);
    return noise4_of(o, K);
}

#ifdef OFDM_PACK_STAMPS   // diagnostic build: s_memtime per item phase, per wave role, summed over the grid
#include <cstdio>
static __device__ unsigned long long g_pack_stamps[4][8];
#define PK_STAMP(k)                                                                  \
    do {                                                                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
        st_acc[k] += t_ - st_t;                                                      \
        st_t = t_;                                                                   \
    } while (0)
#else
#define PK_STAMP(k) do { } while (0)
#endif

// KIND 2: LS estimate from the LTF pair (E spectrum in LDS `ce`, noise from the packed 32-point FFT);
// KIND 0: ideal channel knowledge (AWGN), Z = Y (times (-1)^bin for the C ifft convention, D5).
// CHAN (KIND 2 only): OFDM_CHAN_RAYLEIGH4 applies each frame's 4-tap channel to its clean spectra in the
// group prologue (chan_bin): it does not depend on the SNR point, and the real noise is added after the
// channel (OFDM.c:651 order), so the SNR loop is the AWGN loop with a per-frame E spectrum `fce`.
#define OFDM_RX_PACK_FADE_WAVES 2
#define PACK_SACC_SUB_LS 4  // copies of the block's SNR accumulators, LS receivers (see sacc; at most 4 for the
                            // Rayleigh one, whose two blocks per CU leave room for no more).  A/B (round 4,
                            // profiles/r04/ab): c3 1.236 -> 1.260e10, c5 1.193 -> 1.220e10; 8 copies the same
#define PACK_SACC_SUB 1     // the same for the ideal-CSI receiver (2 copies spill it at its 168-VGPR budget)
// (Wave-reducing the SNR iteration's five counter terms by DPP instead of the 64 same-address LDS atomics per term
// measured negative, round 5, profiles/r05/ab/wave_flush.txt: c2 -5.2 %, c3 -7.0 %, c5 -1.1 % -- the serialised
// atomics run in the LDS pipe beside the VALU stream, the ~70 VALU of the reduction do not.)
template <int KIND, int CONV, int CHAN, bool DUMP>
__global__ __launch_bounds__(256, KIND == 2 ? (CHAN == OFDM_CHAN_RAYLEIGH4 ? OFDM_RX_PACK_FADE_WAVES : OFDM_RX_PACK_WAVES)
                                            : OFDM_RX_PACK_IDEAL_WAVES) void rx_pack_kernel(RxArgs a) {
    constexpr bool FADE = CHAN == OFDM_CHAN_RAYLEIGH4;
    static_assert(!FADE || KIND == 2, "the packed Rayleigh receiver is the LS one");
    // where the next item's L2 warm-up is issued (see the SNR loop)
    constexpr bool WLATE = KIND == 2 && !FADE;
    __shared__ __attribute__((aligned(16))) float4 spec[PACK_PAIRS][2][PK_FRAMES];   // 48 KB: (C[k], C[64-k])
    __shared__ __attribute__((aligned(16))) float4 ce[PACK_PAIRS];                   // LS: FFT((-1)^n 2T[n])
    __shared__ __attribute__((aligned(16))) float4 fce[FADE ? PACK_PAIRS : 1][FADE ? PK_FRAMES : 1];  // 24 KB: H' FFT(2T)
    __shared__ __attribute__((aligned(8))) uint32_t truth[3][PK_SYMS];               // pair-order words
    // flush_lanes' five slots per SNR point; for the first SACC_XQ points SUBN - 1 more copies: lane l adds into
    // copy l % SUBN, so that an SNR iteration's 5 x 64 same-address LDS atomics (the kernel's LDS bank-conflict
    // cycles) spread over SUBN addresses in distinct banks; the copies are summed before the flush
    constexpr int SUBN = KIND != 2 ? PACK_SACC_SUB : FADE ? (PACK_SACC_SUB_LS < 4 ? PACK_SACC_SUB_LS : 4)
                                                      : PACK_SACC_SUB_LS;
    constexpr int SACC_XQ = 16;
    __shared__ unsigned long long sacc[OFDM_MAX_SNR][5];
    __shared__ unsigned long long sacx[SUBN > 1 ? SACC_XQ : 1][SUBN > 1 ? 5 * (SUBN - 1) : 1];
    auto slots = [&](int q, int ln) -> unsigned long long * {
        const int c = ln % SUBN;
        return SUBN > 1 && c > 0 && q < SACC_XQ ? &sacx[q][5 * (c - 1)] : sacc[q];
    };
    __shared__ uint32_t pf_dummy[64];                             // L2 warm-up destination (never read)
    // 8 B of LDS that a pruned option's array held in every measured build (round 6, profiles/r06/README.md): kept,
    // with its per-iteration address, so that the code objects stay byte-identical to the PMC-certified builds
    __shared__ __attribute__((aligned(8))) float2 lds_keep[1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);      // wave-uniform: the SNR loop runs on SGPRs
#ifdef OFDM_PACK_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_t = __builtin_amdgcn_s_memtime();
#endif
    for (int i = tid; i < a.n_snr * 5; i += blockDim.x) (&sacc[0][0])[i] = 0ull;
    if constexpr (SUBN > 1)
        for (int i = tid; i < SACC_XQ * 5 * (SUBN - 1); i += blockDim.x) (&sacx[0][0])[i] = 0ull;
    if constexpr (KIND == 2) {
        // the E window's clean samples 2T[n] (both LTF slots hold T): one spectrum per block
        if (wv == 0) {
            float2 x[64];
            static_for<0, 64>([&](auto nc) {
                constexpr int n = decltype(nc)::value;
                const float2 v = a.ltf[n];
                x[n] = (n & 1) ? make_float2(-2.0f * v.x, -2.0f * v.y) : make_float2(2.0f * v.x, 2.0f * v.y);
            });
            fft64<false>(x);
            if (lane == 0) {
                static_for<0, PACK_PAIRS>([&](auto pc) {
                    constexpr int p = decltype(pc)::value;
                    constexpr int k = pair_bin(p);
                    const float2 c0 = x[digit_rev4(k)], c1 = x[digit_rev4(64 - k)];
                    ce[p] = make_float4(c0.x, c0.y, c1.x, c1.y);
                });
            }
        }
    }
    const int64_t n_groups = (a.n_frames + PK_FRAMES - 1) / PK_FRAMES;
    // Work items: the groups of the full rounds (every block takes gridDim.x-strided groups, all SNR points),
    // then the T tail groups with their SNR points split S ways over up to S T <= gridDim.x blocks, so the
    // last round is not T groups long on T blocks while the rest of the grid idles.  The counters are
    // integer sums: the split does not change them.
    // (32-bit item arithmetic: a launch holds at most 2^23 frames = 2^17 groups)
    const int B = (int)gridDim.x, G = (int)n_groups, R = G / B, T = G - R * B;
    const int S = T > 0 ? max(1, min(4, B / T)) : 1;
    const int n_items = R * B + T * S;
    // Items past the first gridDim.x are handed out one at a time from a.work: during an item's prologue
    // thread 128 fetches the block's next item and wave 2 warms L2 with that item's Tx rows.  Blocks that
    // finish early take more, so the launch ends when the work does, not when the slowest block's static
    // share does.  The next item waits in LDS (read after the SNR loop: nothing 64-bit is held across it).
    __shared__ int next_item;
    for (int w = blockIdx.x; w < n_items; w = __builtin_amdgcn_readfirstlane(next_item)) {
        const bool tail = w >= R * B;
        const int tw = tail ? w - R * B : 0;                           // < T S <= gridDim.x
        const int64_t grp = tail ? R * B + tw / S : w;
        const int sub = tail ? tw % S : 0, ns = tail ? S : 1;
        __syncthreads();                                   // every wave is done with the last group
        PK_STAMP(0);                                       // item-top barrier (waiting for the other waves)
        // group-invariant addresses are re-derived from the thread index here, not held across the SNR
        // loop (they would be the only values spilled)
        int t = tid;
        opaque(t);
        // kernel arguments read where used through an opaque kernarg pointer: hoisted, the 40 words of each
        // TxArgs would be held in SGPRs across the item loop and spill
        using KArgs = const __attribute__((address_space(4))) RxArgs;
        KArgs *ap = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        const bool own_tx = ap->own.n_sym > 0;
        if (own_tx) {
            // this launch's own batch (ofdm_txrx_frames): waves 2-3 build the group's 128 symbols (K2's code,
            // byte-identical), and after the barrier the block reads them back from its XCD's L2 like a batch
            // built by an earlier launch.  Every item of a group builds it (a tail group's SNR subsets run on
            // several blocks): the duplicate stores write identical bytes.
            if (t >= PK_SYMS) {
                const int64_t sidx = grp * PK_SYMS + (t - PK_SYMS);
                if (sidx < ap->own.n_sym) {
                    if (ap->own_conv == OFDM_CONV_C) tx_symbol<OFDM_CONV_C>(ap->own, sidx);
                    else tx_symbol<OFDM_CONV_MATLAB>(ap->own, sidx);
                }
            }
            __syncthreads();
        }
        if (t < PK_SYMS) {
            clean_spectrum(a, grp * PK_SYMS + t, &spec[0][t & 1][t >> 1]);
        } else {
            const int j = t - PK_SYMS;
            const uint32_t *src = a.bits + 7 * a.pitch + grp * PK_SYMS + j;
            truth[0][j] = src[0];
            truth[1][j] = src[a.pitch];
            truth[2][j] = src[2 * a.pitch];
            if (j < 64) {                                  // wave 2: the next item
                int nx = 0;
                if (j == 0) nx = B + (int)atomicAdd(a.work, 1ull);
                nx = __builtin_amdgcn_readlane(nx, 0);          // lane 0 (j == 0) fetched it
                if (j == 0) next_item = nx;
                // warm L2 with the next item's group (64 rows x 1 KB: one 4-byte LDS-DMA read per 128-B
                // line, into a dummy LDS word), so the next prologue's loads hit L2 instead of HBM (not when
                // the launch builds its own batch: those rows are written by the next item itself)
                if (nx < n_items && !own_tx && !WLATE) {
                    const int64_t ng = nx < R * B ? nx : R * B + (nx - R * B) / S;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int line = j + 64 * i;                       // 0..511
                        const float2 *p = a.tx + (int64_t)(16 + (line >> 3)) * a.pitch + ng * PK_SYMS + (line & 7) * 16;
                        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)p,
                                                         (__attribute__((address_space(3))) void *)pf_dummy, 4, 0, 0);
                    }
                }
            }
            // the next chunk's Tx batch (ofdm_set_next_tx), one symbol per lane: group gg of this launch's
            // sub-0 item builds the next batch's symbols [128 gg', 128 gg' + 128) for gg' = gg, gg + G, ...
            if (ap->nx.n_sym > 0 && sub == 0) {
                for (int64_t sidx = grp * PK_SYMS + j; sidx < ap->nx.n_sym; sidx += (int64_t)G * PK_SYMS) {
                    if (ap->nx_conv == OFDM_CONV_C) tx_symbol<OFDM_CONV_C>(ap->nx, sidx);
                    else tx_symbol<OFDM_CONV_MATLAB>(ap->nx, sidx);
                }
            }
            if constexpr (FADE) {      // the group's channel responses, a frame's 24 pairs split over waves 2 / 3
                const int fr = j & 63;
                const uint64_t ff = a.first_frame + (uint64_t)(grp * PK_FRAMES + fr);
                float2 h[4];
                channel_taps((uint32_t)ff, (uint32_t)(ff >> 32), a.k0, a.k1, h);
                if (j < 64) chan_pairs<0>(h, &fce[0][fr]);
                else chan_pairs<1>(h, &fce[0][fr]);
            }
        }
        PK_STAMP(1);                                       // prologue work
        __syncthreads();
        PK_STAMP(2);                                       // prologue barrier
        if constexpr (FADE) {
            // faded spectra: C <- H' C for both data symbols, and fce <- H' FFT(2T) (the frame's LS reference);
            // one (pair, frame) per thread and step, so each H' is read and overwritten by one thread
            for (int it = t; it < PACK_PAIRS * PK_FRAMES; it += 256) {
                const int p = it >> 6, fr = it & 63;
                const float4 H = fce[p][fr], c0 = spec[p][0][fr], c1 = spec[p][1][fr], e = ce[p];
                const float2 Hk = make_float2(H.x, H.y), Hm = make_float2(H.z, H.w);
                float2 u = cmul(Hk, make_float2(c0.x, c0.y)), v = cmul(Hm, make_float2(c0.z, c0.w));
                spec[p][0][fr] = make_float4(u.x, u.y, v.x, v.y);
                u = cmul(Hk, make_float2(c1.x, c1.y)); v = cmul(Hm, make_float2(c1.z, c1.w));
                spec[p][1][fr] = make_float4(u.x, u.y, v.x, v.y);
                u = cmul(Hk, make_float2(e.x, e.y)); v = cmul(Hm, make_float2(e.z, e.w));
                fce[p][fr] = make_float4(u.x, u.y, v.x, v.y);
            }
            __syncthreads();
        }
        PK_STAMP(3);                                       // Rayleigh: faded spectra
        const int64_t fl = grp * PK_FRAMES + lane;
        const bool valid = fl < a.n_frames;
        const uint64_t f = a.first_frame + (uint64_t)fl;
        for (int q = wv + 4 * sub; q < a.n_snr; q += 4 * ns) {
            // LS AWGN: wave 2 warms L2 with the next item's rows at the start of its last SNR iteration, one
            // iteration before the next prologue reads them (warmed in the prologue, a whole item earlier, most
            // lines were evicted again: 64 blocks per XCD warm 4 MB into its 4 MB L2)
            if constexpr (WLATE) {
                if (wv == 2 && q + 4 * ns >= a.n_snr) {
                    const int nx = __builtin_amdgcn_readfirstlane(next_item);
                    using KArgsW = const __attribute__((address_space(4))) RxArgs;
                    KArgsW *apw = (KArgsW *)__builtin_amdgcn_kernarg_segment_ptr();
                    if (nx < n_items && apw->own.n_sym == 0) {
                        const int64_t ng = nx < R * B ? nx : R * B + (nx - R * B) / S;
                        const int ln = lane;
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const int line = ln + 64 * i;                      // 0..511
                            const float2 *p = a.tx + (int64_t)(16 + (line >> 3)) * a.pitch + ng * PK_SYMS + (line & 7) * 16;
                            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)p,
                                                             (__attribute__((address_space(3))) void *)pf_dummy, 4, 0, 0);
                        }
                    }
                }
            }
            uint32_t flo = (uint32_t)f, fhi = (uint32_t)(f >> 32);
            opaque(flo); opaque(fhi);
            const float sigma = a.sigma[q];
            const uint32_t qs = STREAM_NOISE | (uint32_t)(a.q_base + q);
            const PhiloxHead hd = philox_head(flo, fhi, qs, a.k1);
            // ---- LTF pair noise (LS): e[n] = sqrt2 sigma x Gaussian 192 + n (block 48 + n/4), packed as
            // z[m] = e'[2m] + j e'[2m+1] with e'[n] = (-1)^n e[n]; radix-2 stage fused, then two dif4<16>
            float2 z[64];      // z[0..31] used
            float2 ee[PACK_PAIRS];
            lf2 *keep = (lf2 *)&lds_keep[0];
            opaque(keep);
            if constexpr (KIND == 2) {
                const float KE = noise_k(sigma * 1.41421356237309504880f);
                static_for<0, 4>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    uint32_t tg = 48u + 2 * i;
                    opaque(tg);
                    // blocks b = 2i, 2i+1 (z[4i..4i+3]) and b + 8 (z[4i+16..4i+19])
                    static_for<0, 2>([&](auto hc) {
                        constexpr int h = decltype(hc)::value;
                        const Noise4 lo = pack_noise(hd, tg + h, a.k0, a.k1, KE);
                        const Noise4 hi = pack_noise(hd, tg + 8 + h, a.k0, a.k1, KE);
                        constexpr int m = 4 * i + 2 * h;
                        z[m] = make_float2(lo.r0 * lo.c0, -(lo.r0 * lo.s0));
                        z[m + 1] = make_float2(lo.r1 * lo.c1, -(lo.r1 * lo.s1));
                        z[m + 16] = make_float2(hi.r0 * hi.c0, -(hi.r0 * hi.s0));
                        z[m + 17] = make_float2(hi.r1 * hi.c1, -(hi.r1 * hi.s1));
                    });
                    static_for<0, 4>([&](auto jc) {
                        constexpr int j = 4 * i + decltype(jc)::value;
                        const float2 u = z[j], v = z[j + 16];
                        z[j] = cadd(u, v);
                        z[j + 16] = twiddle<2 * j, false>(csub(u, v));     // W32^j
                    });
                    sched_fence();
                });
                dif4<false, 16, 0>(z);
                dif4<false, 16, 16>(z);
                // E'[k] = (Z[k] + conj Z[-k]) / 2 - j W64^k (Z[k] - conj Z[-k]) / 2 (Z indices mod 32), kept
                // as 2 E'[k] per pair (48 VGPRs instead of the 62 of Z); E'[64 - k] = conj E'[k]
                static_for<0, PACK_PAIRS>([&](auto pc) {
                    constexpr int p = decltype(pc)::value;
                    constexpr int k = pair_bin(p);
                    const float2 P = z[pos32(k)], Qv = z[pos32(32 - k)];
                    const float2 F = make_float2(P.x + Qv.x, P.y - Qv.y);
                    const float2 H = twiddle<k, false>(make_float2(P.x - Qv.x, P.y + Qv.y));
                    ee[p] = make_float2(F.x + H.y, F.y - H.x);
                });
                sched_fence();
            }
            // ---- data windows: x[n] = (-1)^n (d0[n] + j d1[n]) fused with the first radix-4 stage.
            // Gaussian t of the frame's stream is sample t of the frame timeline: D0 at
            // t = 336 + n (Philox block 84 + n/4), D1 at t = 416 + n (block 104 + n/4).
            const float K = noise_k(sigma);
            float2 x[64];
            static_for<0, 4>([&](auto gc) {
                constexpr int g = decltype(gc)::value;
                uint32_t tg = 84u + g;
                opaque(tg);
                static_for<0, 4>([&](auto Qc) {
                    constexpr int Q = decltype(Qc)::value;
                    const Noise4 n0 = pack_noise(hd, tg + 4 * Q, a.k0, a.k1, K);
                    const Noise4 n1 = pack_noise(hd, tg + 20 + 4 * Q, a.k0, a.k1, K);
                    const float d0[4] = {n0.r0 * n0.c0, n0.r0 * n0.s0, n0.r1 * n0.c1, n0.r1 * n0.s1};
                    const float d1[4] = {n1.r0 * n1.c0, n1.r0 * n1.s0, n1.r1 * n1.c1, n1.r1 * n1.s1};
                    static_for<0, 4>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        x[16 * Q + 4 * g + i] = (i & 1) ? make_float2(-d0[i], -d1[i]) : make_float2(d0[i], d1[i]);
                    });
                    if constexpr (Q % PACK_GEN_SPLIT == PACK_GEN_SPLIT - 1 && Q < 3) sched_fence();
                });
                static_for<0, 4>([&](auto ic) { dif_stage1<false, 4 * g + decltype(ic)::value>(x); });
                sched_fence();
            });
            // ---- bin pairs: noise split, clean spectra, estimate, equaliser, demap of both data symbols
            float2 *deq0 = nullptr, *deq1 = nullptr;
            uint32_t *dbit0 = nullptr, *dbit1 = nullptr;
            if constexpr (DUMP) {
                if (valid) {
                    const int64_t r0 = ((int64_t)q * a.dump_frames + fl) * 2;
                    deq0 = a.dump_eq + r0 * 48; deq1 = deq0 + 48;
                    dbit0 = a.dump_bits + r0 * 3; dbit1 = dbit0 + 3;
                }
            }
            uint32_t db0[3] = {0u, 0u, 0u}, db1[3] = {0u, 0u, 0u};
            lcf4 *sp = (lcf4 *)&spec[0][0][lane];
            lcu2 *tw = (lcu2 *)&truth[0][2 * lane];
            lcf4 *fp = (lcf4 *)&fce[0][FADE ? lane : 0];   // per-iteration address: the loads stay in the loop
            opaque(sp); opaque(tw);
            if constexpr (FADE) opaque(fp);
            uint32_t sm;
            asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(sm));
            float evm = 0.f;
            uint32_t em = 0u, be = 0u, ax = 0u, t0 = 0u, t1 = 0u;
            // LDS operands of a bin pair (both clean spectra and, LS, the E spectrum), loaded PF pairs ahead of
            // their use so that the read latency is covered by the pairs in between (the fences every
            // PACK_FENCE_PAIRS pairs keep the loads where they are written)
            constexpr int PF = KIND == 2 && !FADE ? PACK_PF : 0;
            f4v pc0[PF + 1], pc1[PF + 1];
            float4 pe4[PF + 1];
            auto load_pair = [&](auto pc) {
                constexpr int p = decltype(pc)::value;
                if constexpr (p < PACK_PAIRS) {
                    constexpr int slot = p % (PF + 1);
                    pc0[slot] = sp[p * 2 * PK_FRAMES];
                    pc1[slot] = sp[(p * 2 + 1) * PK_FRAMES];
                    if constexpr (KIND == 2) {
                        if constexpr (FADE) {
                            const f4v v = fp[p * PK_FRAMES];
                            pe4[slot] = make_float4(v.x, v.y, v.z, v.w);
                        } else {
                            pe4[slot] = ce[p];
                        }
                    }
                }
            };
            if constexpr (PF > 0) static_for<0, PF>(load_pair);
            auto pair = [&](auto pc) {
                constexpr int p = decltype(pc)::value;
                constexpr int k = pair_bin(p), k2 = 64 - k;
                if constexpr ((p & 7) == 0) {
                    const u2v tt = tw[(p >> 3) * (PK_SYMS / 2)];
                    t0 = tt.x; t1 = tt.y;
                }
                if constexpr (PF > 0) load_pair(std::integral_constant<int, p + PF>{});
                constexpr int slot = p % (PF + 1);
                const float2 Zk = x[digit_rev4(k)], Zm = x[digit_rev4(k2)];
                const float2 A = make_float2(Zk.x + Zm.x, Zk.y - Zm.y), B = make_float2(Zk.x - Zm.x, Zk.y + Zm.y);
                if constexpr (PF == 0) load_pair(pc);
                const f4v c0 = pc0[slot], c1 = pc1[slot];
                // Y_d = C_d + N_d:  N0[k] = A/2, N0[k'] = conj(A)/2, N1[k] = -j B/2, N1[k'] = conj(N1[k])
                const float2 y0k = make_float2(fmaf(0.5f, A.x, c0.x), fmaf(0.5f, A.y, c0.y));
                const float2 y0m = make_float2(fmaf(0.5f, A.x, c0.z), fmaf(-0.5f, A.y, c0.w));
                const float2 y1k = make_float2(fmaf(0.5f, B.y, c1.x), fmaf(-0.5f, B.x, c1.y));
                const float2 y1m = make_float2(fmaf(0.5f, B.y, c1.z), fmaf(0.5f, B.x, c1.w));
                float2 u0k, u0m, u1k, u1m;
                float rk = 0.f, rm = 0.f;
                if constexpr (KIND == 2) {
                    const float ex = ee[p].x, ey = ee[p].y;
                    const float4 e4 = pe4[slot];
                    const float2 Sk = make_float2(fmaf(0.5f, ex, e4.x), fmaf(0.5f, ey, e4.y));
                    const float2 Sm = make_float2(fmaf(0.5f, ex, e4.z), fmaf(-0.5f, ey, e4.w));
                    rk = __builtin_amdgcn_rcpf(fmaf(Sk.x, Sk.x, Sk.y * Sk.y));
                    rm = __builtin_amdgcn_rcpf(fmaf(Sm.x, Sm.x, Sm.y * Sm.y));
                    // Z = Y / (0.5 Lf S) = 2 Lf Y conj(S) / |S|^2: u = Lf Y conj(S), g = 2 r
                    u0k = cscale(cmulc(y0k, Sk), (float)ltf_sign(k));
                    u1k = cscale(cmulc(y1k, Sk), (float)ltf_sign(k));
                    u0m = cscale(cmulc(y0m, Sm), (float)ltf_sign(k2));
                    u1m = cscale(cmulc(y1m, Sm), (float)ltf_sign(k2));
                } else {
                    constexpr float cs = (CONV == OFDM_CONV_C && (k & 1)) ? -1.0f : 1.0f;   // k, k2 same parity
                    u0k = cscale(y0k, cs); u0m = cscale(y0m, cs); u1k = cscale(y1k, cs); u1m = cscale(y1m, cs);
                }
                demap_bin<KIND, DUMP>(u0k, rk, t0, sm, evm, em, data_index(k), deq0, db0);
                demap_bin<KIND, DUMP>(u0m, rm, t0, sm, evm, em, data_index(k2), deq0, db0);
                demap_bin<KIND, DUMP>(u1k, rk, t1, sm, evm, em, data_index(k), deq1, db1);
                demap_bin<KIND, DUMP>(u1m, rm, t1, sm, evm, em, data_index(k2), deq1, db1);
                if constexpr ((p & 3) == 3) {
                    // 16 decisions: im errors at even bit positions, re errors at odd
                    ax += __popc(em);
                    be += __popc(em & 0x55555555u) + __popc((em ^ (em >> 1)) & 0x55555555u);
                    em = 0u;
                }
                // pin the per-bin EVM terms here: left alone, LLVM sinks the whole fma chain to its
                // single use after the last pair and keeps every bin's u' alive until then
                opaque(evm);
                if constexpr (p % PACK_FENCE_PAIRS == PACK_FENCE_PAIRS - 1) sched_fence();
            };
            dif_sub16<false, 0>(x);
            static_for<0, 6>(pair);
            sched_fence();
            dif_sub16<false, 2>(x);
            static_for<6, 13>(pair);
            sched_fence();
            dif_sub16<false, 1>(x);
            dif_sub16<false, 3>(x);
            static_for<13, 24>(pair);
            if constexpr (DUMP) {
                if (dbit0) {
                    dbit0[0] = db0[0]; dbit0[1] = db0[1]; dbit0[2] = db0[2];
                    dbit1[0] = db1[0]; dbit1[1] = db1[1]; dbit1[2] = db1[2];
                }
            }
            FrameAcc acc;
            frame_metrics(acc, KIND == 2 ? 4.0f * evm : evm, be, ax);
            flush_lanes(acc, valid, slots(q, lane));
        }
        PK_STAMP(4);                                     // SNR loop
    }
    if constexpr (SUBN > 1) {       // fold the copies into sacc
        __syncthreads();
        for (int i = tid; i < min(a.n_snr, SACC_XQ) * 5; i += 256) {
            const int q = i / 5, k = i % 5;
            unsigned long long v = sacc[q][k];
#pragma unroll
            for (int c = 1; c < SUBN; ++c) v += sacx[q][5 * (c - 1) + k];
            sacc[q][k] = v;
        }
    }
    block_flush(a, sacc, tid);
    PK_STAMP(5);                                           // block flush
#ifdef OFDM_PACK_STAMPS
    if (lane == 0)
        for (int k = 0; k < 6; ++k) atomicAdd(&g_pack_stamps[wv][k], st_acc[k]);
#endif
}

template <int KIND, int CONV, int CHAN = OFDM_CHAN_AWGN>
static void launch_pack_t(hipStream_t st, const RxArgs &a, bool dump, unsigned grid) {
    if (dump) hipLaunchKernelGGL((rx_pack_kernel<KIND, CONV, CHAN, true>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((rx_pack_kernel<KIND, CONV, CHAN, false>), dim3(grid), dim3(256), 0, st, a);
#ifdef OFDM_PACK_STAMPS
    // cumulative over the process's launches: wave 0 (clean spectra) and wave 2 (Tx / warm-up) roles
    unsigned long long hs[4][8];
    if (hipStreamSynchronize(st) == hipSuccess && hipMemcpyFromSymbol(hs, HIP_SYMBOL(g_pack_stamps), sizeof hs) == hipSuccess) {
        static const char *names[6] = {"item-top barrier", "prologue work", "prologue barrier", "faded spectra",
                                       "SNR loop", "block flush"};
        for (int w : {0, 2}) {
            double tot = 0;
            for (int k = 0; k < 6; ++k) tot += (double)hs[w][k];
            fprintf(stderr, "pack stamp wave %d:", w);
            for (int k = 0; k < 6; ++k) fprintf(stderr, " %s %.2f%%;", names[k], 100.0 * (double)hs[w][k] / tot);
            fprintf(stderr, "\n");
        }
    }
#endif
}

template <const void *(*K)()>
static int pack_grid(int64_t n_frames, int device) {
    const int64_t need = (n_frames + PK_FRAMES - 1) / PK_FRAMES;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K(), 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
    const int64_t cap = (int64_t)per_cu * cus;
    const int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
}

#ifdef OFDM_RXPACK_IDEAL_TU
// The ideal-CSI receivers (KIND 0) are instantiated in their own translation unit (ofdm_rxpack_ideal.hip),
// compiled with LLVM's default scheduler: with the group prologue's Tx builds, max-ILP scheduling of the
// 168-VGPR (3 waves/SIMD) receiver spills, the default one fits (163 VGPRs).
static const void *ideal_kernel() { return reinterpret_cast<const void *>(&rx_pack_kernel<0, OFDM_CONV_C, OFDM_CHAN_AWGN, false>); }

void launch_rx_pack_ideal(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid) {
    if (cfg.conv == OFDM_CONV_C) launch_pack_t<0, OFDM_CONV_C>(st, a, dump, grid);
    else launch_pack_t<0, OFDM_CONV_MATLAB>(st, a, dump, grid);
}

int rx_pack_ideal_grid(int64_t n_frames, int device) { return pack_grid<ideal_kernel>(n_frames, device); }
#else
// Real-noise sweeps: AWGN with either estimator, and the 4-tap Rayleigh channel with the LS estimator
// (the ideal-CSI Rayleigh ZF and every complex-noise sweep run the {E, D0, D1} / ideal receivers).
bool rx_pack_applies(const ofdm_cfg &cfg) {
    if (cfg.noise != OFDM_NOISE_REAL) return false;
    if (cfg.channel == OFDM_CHAN_RAYLEIGH4) return cfg.est == OFDM_EST_LS;
    return cfg.channel == OFDM_CHAN_AWGN;
}

void launch_rx_pack(hipStream_t st, const RxArgs &a, const ofdm_cfg &cfg, bool dump, unsigned grid) {
    if (cfg.est == OFDM_EST_LS && cfg.channel == OFDM_CHAN_RAYLEIGH4)
        launch_pack_t<2, OFDM_CONV_C, OFDM_CHAN_RAYLEIGH4>(st, a, dump, grid);           // conv via a.ltf
    else if (cfg.est == OFDM_EST_LS) launch_pack_t<2, OFDM_CONV_C>(st, a, dump, grid);
    else launch_rx_pack_ideal(st, a, cfg, dump, grid);
}

static const void *ls_kernel() { return reinterpret_cast<const void *>(&rx_pack_kernel<2, OFDM_CONV_C, OFDM_CHAN_AWGN, false>); }
static const void *fade_kernel() {
    return reinterpret_cast<const void *>(&rx_pack_kernel<2, OFDM_CONV_C, OFDM_CHAN_RAYLEIGH4, false>);
}

int rx_pack_grid(const ofdm_cfg &cfg, int64_t n_frames, int device) {
    if (cfg.est != OFDM_EST_LS) return rx_pack_ideal_grid(n_frames, device);
    return cfg.channel == OFDM_CHAN_RAYLEIGH4 ? pack_grid<fade_kernel>(n_frames, device)
                                              : pack_grid<ls_kernel>(n_frames, device);
}
#endif

}  // namespace ofdm
