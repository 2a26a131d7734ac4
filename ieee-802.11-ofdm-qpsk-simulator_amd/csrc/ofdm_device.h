// ofdm_device.h -- device building blocks for the gfx950 OFDM Monte-Carlo kernels.
//
//  * Philox4x32-10 counter-based RNG (Salmon et al., SC'11; Random123 constants), keyed by the
//    64-bit seed; the stream/counter layout is DESIGN.md §3 (shared with oracle/ofdm_oracle.c).
//  * Box-Muller on the hardware transcendentals (v_log_f32, v_sqrt_f32, v_sin/v_cos_f32 which
//    take revolutions, so 2*pi*u needs no range reduction).
//  * a fully unrolled radix-4 decimation-in-frequency 64-point FFT held in one lane's VGPRs
//    (x[64] indexed only by compile-time constants), digit-reversed output.  One lane owns one
//    OFDM symbol, so no cross-lane traffic is needed on the hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "twiddle64.h"

namespace ofdm {

// ------------------------------------------------------------------ compile-time loops
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Hide a value from the optimiser for one program point.  Used inside the per-SNR loop so that
// loop-invariant work (64 load addresses, 96 truth-symbol selects, the first Philox round) is
// recomputed each iteration instead of being hoisted and held in ~200 extra VGPRs.
template <typename T>
__device__ __forceinline__ void opaque(T &v) { asm volatile("" : "+v"(v)); }

// ------------------------------------------------------------------ complex helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
    return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -a.x * b.y));
}

// ------------------------------------------------------------------ Philox4x32-10
constexpr uint32_t PHILOX_M0 = 0xD2511F53u, PHILOX_M1 = 0xCD9E8D57u;
constexpr uint32_t PHILOX_W0 = 0x9E3779B9u, PHILOX_W1 = 0xBB67AE85u;
// stream tags in counter word 3
constexpr uint32_t STREAM_BITS = 0xB1750000u;
constexpr uint32_t STREAM_NOISE = 0x5A000000u;
constexpr uint32_t STREAM_CHAN = 0xC4A00000u;
constexpr uint32_t STREAM_START = 0x5B000000u;

__device__ __forceinline__ uint4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                          uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)PHILOX_M0 * c0;   // v_mad_u64_u32
        const uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        // 3-input XOR in one v_bitop3_b32 (truth table 0x96), key words from SGPRs
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    return make_uint4(c0, c1, c2, c3);
}

// philox10 for many calls that share counter words c0, c1 (the frame) and c3 (stream | SNR index)
// and differ only in c2: round 1's c0 product does not depend on c2, so philox_head() computes it
// once and philox10_c2() does the c2 half of round 1 and rounds 2..10 (same output as philox10).
struct PhiloxHead { uint32_t c1, n2, c3; };
__device__ __forceinline__ PhiloxHead philox_head(uint32_t c0, uint32_t c1, uint32_t c3, uint32_t k1) {
    const uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    return {c1, (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96), (uint32_t)p0};
}
__device__ __forceinline__ uint4 philox10_c2(const PhiloxHead &h, uint32_t c2, uint32_t k0, uint32_t k1) {
    const uint64_t p1r = (uint64_t)PHILOX_M1 * c2;
    uint32_t c0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1r >> 32), h.c1, k0, 0x96);
    uint32_t c1 = (uint32_t)p1r, c3 = h.c3;
    c2 = h.n2;
    k0 += PHILOX_W0; k1 += PHILOX_W1;
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        const uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    return make_uint4(c0, c1, c2, c3);
}

// Round keys k0 + r W0, k1 + r W1 (r = 0..9) held in VGPRs: a v_bitop3_b32 with an SGPR operand issues
// at the slow rate, with three VGPR operands at the fast rate.  Built once per kernel
// (asm v_mov: never rematerialised into SGPR form); 20 VGPRs.
struct PhiloxKeysV {
    uint32_t k0[10], k1[10];
    __device__ __forceinline__ void init(uint32_t s0, uint32_t s1) {
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            asm volatile("v_mov_b32 %0, %1" : "=v"(k0[r]) : "s"(s0 + (uint32_t)r * PHILOX_W0));
            asm volatile("v_mov_b32 %0, %1" : "=v"(k1[r]) : "s"(s1 + (uint32_t)r * PHILOX_W1));
        }
    }
};
// philox10_c2 with the round keys in VGPRs (same output)
__device__ __forceinline__ uint4 philox10_c2(const PhiloxHead &h, uint32_t c2, const PhiloxKeysV &k) {
    const uint64_t p1r = (uint64_t)PHILOX_M1 * c2;
    uint32_t c0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1r >> 32), h.c1, k.k0[0], 0x96);
    uint32_t c1 = (uint32_t)p1r, c3 = h.c3;
    c2 = h.n2;
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        const uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k.k0[r], 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k.k1[r], 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    return make_uint4(c0, c1, c2, c3);
}

// philox10_c2 for NB blocks at once with the round keys in VGPRs (same outputs), round-major: the NB blocks'
// multiply chains interleave (ILP 2 NB) instead of running one block after another
template <int NB>
__device__ __forceinline__ void philox10_c2_multi(const PhiloxHead &h, const uint32_t (&c2in)[NB], const PhiloxKeysV &k,
                                                  uint4 (&out)[NB]) {
    uint32_t c0[NB], c1[NB], c2[NB], c3[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint64_t p1r = (uint64_t)PHILOX_M1 * c2in[b];
        c0[b] = __builtin_amdgcn_bitop3_b32((uint32_t)(p1r >> 32), h.c1, k.k0[0], 0x96);
        c1[b] = (uint32_t)p1r; c2[b] = h.n2; c3[b] = h.c3;
    }
#pragma unroll
    for (int r = 1; r < 10; ++r) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint64_t p0 = (uint64_t)PHILOX_M0 * c0[b];
            const uint64_t p1 = (uint64_t)PHILOX_M1 * c2[b];
            const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1[b], k.k0[r], 0x96);
            const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3[b], k.k1[r], 0x96);
            c0[b] = n0; c1[b] = (uint32_t)p1; c2[b] = n2; c3[b] = (uint32_t)p0;
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) out[b] = make_uint4(c0[b], c1[b], c2[b], c3[b]);
}

// philox10_c2 for NB blocks at once (same outputs), round keys in VGPRs: a v_bitop3_b32 with an SGPR
// operand issues at the slow rate, one with three VGPRs at the fast rate.  The keys
// are moved to VGPRs once and advanced round by round with v_add (literal W0 / W1), shared by the NB
// blocks; opaque() keeps the nine round keys from being formed up front (2 live VGPRs, not 18).
template <int NB>
__device__ __forceinline__ void philox10_c2_vk(const PhiloxHead &h, const uint32_t (&c2in)[NB], uint32_t k0,
                                               uint32_t k1, uint4 (&out)[NB]) {
    uint32_t kv0, kv1;
    asm volatile("v_mov_b32 %0, %1" : "=v"(kv0) : "s"(k0));
    asm volatile("v_mov_b32 %0, %1" : "=v"(kv1) : "s"(k1));
    uint32_t c0[NB], c1[NB], c2[NB], c3[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint64_t p1r = (uint64_t)PHILOX_M1 * c2in[b];
        c0[b] = __builtin_amdgcn_bitop3_b32((uint32_t)(p1r >> 32), h.c1, kv0, 0x96);
        c1[b] = (uint32_t)p1r; c2[b] = h.n2; c3[b] = h.c3;
    }
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        kv0 += PHILOX_W0; kv1 += PHILOX_W1;
        opaque(kv0); opaque(kv1);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint64_t p0 = (uint64_t)PHILOX_M0 * c0[b];
            const uint64_t p1 = (uint64_t)PHILOX_M1 * c2[b];
            const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1[b], kv0, 0x96);
            const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3[b], kv1, 0x96);
            c0[b] = n0; c1[b] = (uint32_t)p1; c2[b] = n2; c3[b] = (uint32_t)p0;
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) out[b] = make_uint4(c0[b], c1[b], c2[b], c3[b]);
}

// The Box-Muller angle of a Philox word x, in revolutions (v_sin / v_cos take revolutions).
__device__ __forceinline__ float bm_angle(uint32_t x) {
    return (float)x * 0x1p-32f;
}

// Box-Muller pair.  u1 = fma((float)x1, 2^-32, 2^-33) in (0, 1] (tail to 6.7 sigma);
// u2 = (float)x2 * 2^-32 in revolutions.  Same quantisation as oracle/ofdm_oracle.c:bm_pair.
__device__ __forceinline__ float2 box_muller(uint32_t x1, uint32_t x2) {
    const float u1 = fmaf((float)x1, 0x1p-32f, 0x1p-33f);
    const float u2 = bm_angle(x2);
    // -2 ln(u1) = -2 ln(2) log2(u1)
    const float r = __builtin_amdgcn_sqrtf(-1.38629436111989061883f * __builtin_amdgcn_logf(u1));
    return make_float2(r * __builtin_amdgcn_cosf(u2), r * __builtin_amdgcn_sinf(u2));
}

// The same four draws scaled by sigma, left as radius and angle terms so that each noisy sample
// is one fma: sigma z = r (cos | sin), r = sqrt(K log2 u1) with K = -2 ln(2) sigma^2 folded under
// the square root (sigma sqrt(-2 ln u1) = sqrt(-2 ln 2 sigma^2 log2 u1)).
struct Noise4 { float r0, c0, s0, r1, c1, s1; };   // sigma (z0, z1, z2, z3) = (r0 c0, r0 s0, r1 c1, r1 s1)
__device__ __forceinline__ float noise_k(float sigma) { return -1.38629436111989061883f * sigma * sigma; }

// four N(0,1) draws of one Philox block
struct Gauss4 { float z[4]; };
__device__ __forceinline__ Gauss4 gauss4_of(uint4 o) {
    const float2 a = box_muller(o.x, o.y), b = box_muller(o.z, o.w);
    Gauss4 g;
    g.z[0] = a.x; g.z[1] = a.y; g.z[2] = b.x; g.z[3] = b.y;
    return g;
}
__device__ __forceinline__ Gauss4 gauss4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                         uint32_t k0, uint32_t k1) {
    return gauss4_of(philox10(c0, c1, c2, c3, k0, k1));
}

__device__ __forceinline__ Noise4 noise4_of(uint4 o, float K) {
    const float u1a = fmaf((float)o.x, 0x1p-32f, 0x1p-33f), u2a = bm_angle(o.y);
    const float u1b = fmaf((float)o.z, 0x1p-32f, 0x1p-33f), u2b = bm_angle(o.w);
    Noise4 n;
    n.r0 = __builtin_amdgcn_sqrtf(K * __builtin_amdgcn_logf(u1a));
    n.r1 = __builtin_amdgcn_sqrtf(K * __builtin_amdgcn_logf(u1b));
    n.c0 = __builtin_amdgcn_cosf(u2a); n.s0 = __builtin_amdgcn_sinf(u2a);
    n.c1 = __builtin_amdgcn_cosf(u2b); n.s1 = __builtin_amdgcn_sinf(u2b);
    return n;
}

// ------------------------------------------------------------------ twiddles
// multiply by e^{-j 2 pi E / 64} (forward) or e^{+j 2 pi E / 64} (inverse); trivial cases free
template <int E, bool INV>
__device__ __forceinline__ float2 twiddle(float2 a) {
    constexpr int e = ((E % 64) + 64) % 64;
    if constexpr (e == 0) {
        return a;
    } else if constexpr (e == 32) {
        return make_float2(-a.x, -a.y);
    } else if constexpr ((e == 16 && !INV) || (e == 48 && INV)) {   // * (-j)
        return make_float2(a.y, -a.x);
    } else if constexpr ((e == 48 && !INV) || (e == 16 && INV)) {   // * (+j)
        return make_float2(-a.y, a.x);
    } else {
        constexpr float wr = kCos64[e];
        constexpr float wi = INV ? kSin64[e] : -kSin64[e];
        return make_float2(fmaf(a.x, wr, -a.y * wi), fmaf(a.x, wi, a.y * wr));
    }
}

// ------------------------------------------------------------------ radix-4 DIF 64-point FFT
// x[k] natural order in; out: bin k at position digit_rev4(k).  Unnormalised.
// Forward: X[k] = sum x[n] e^{-j2pi kn/64}; inverse: e^{+j...}.
// The transform is exposed in pieces so callers can bound register live ranges:
//   dif_bfly<INV, N, B, j>  one radix-4 butterfly (+ twiddles) of the stage of span N at offset B
//   dif_stage1<INV, j>      butterfly j (0..15) of the first 64-point stage
//   dif_sub16<INV, R>       the remaining two stages of sub-block R (positions 16R..16R+15);
//                           afterwards bins k with (k & 3) == R are final.
template <bool INV, int N, int B, int j>
__device__ __forceinline__ void dif_bfly(float2 (&x)[64]) {
    constexpr int Q = N / 4;
    constexpr int S = 64 / N;
    const float2 a = x[B + j], b = x[B + j + Q], c = x[B + j + 2 * Q], d = x[B + j + 3 * Q];
    const float2 t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
    float2 y1, y3;
    if constexpr (!INV) {
        y1 = make_float2(t1.x + t3.y, t1.y - t3.x);   // t1 - j t3
        y3 = make_float2(t1.x - t3.y, t1.y + t3.x);   // t1 + j t3
    } else {
        y1 = make_float2(t1.x - t3.y, t1.y + t3.x);
        y3 = make_float2(t1.x + t3.y, t1.y - t3.x);
    }
    x[B + j] = cadd(t0, t2);
    x[B + j + Q] = twiddle<j * S, INV>(y1);
    x[B + j + 2 * Q] = twiddle<2 * j * S, INV>(csub(t0, t2));
    x[B + j + 3 * Q] = twiddle<3 * j * S, INV>(y3);
}

template <bool INV, int N, int B>
__device__ __forceinline__ void dif4(float2 (&x)[64]) {
    if constexpr (N >= 4) {
        constexpr int Q = N / 4;
        static_for<0, Q>([&](auto jc) { dif_bfly<INV, N, B, decltype(jc)::value>(x); });
        dif4<INV, Q, B>(x);
        dif4<INV, Q, B + Q>(x);
        dif4<INV, Q, B + 2 * Q>(x);
        dif4<INV, Q, B + 3 * Q>(x);
    }
}

template <bool INV, int j>
__device__ __forceinline__ void dif_stage1(float2 (&x)[64]) { dif_bfly<INV, 64, 0, j>(x); }
template <bool INV, int R>
__device__ __forceinline__ void dif_sub16(float2 (&x)[64]) { dif4<INV, 16, 16 * R>(x); }

// this lane's index re-derived where it is used (v_mbcnt, volatile: never hoisted), so that a kernel at a
// tight register budget does not hold the work-item id in a VGPR across its long loops
__device__ __forceinline__ int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

// global-address-space views (keep loads global_* after opaque(), which erases provenance).
// Native clang vectors, not float2 (HIP_vector_type's members are not address-space qualified).
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f2v gcf2;
typedef __attribute__((address_space(1))) f2v gf2;
__device__ __forceinline__ float2 gld(gcf2 *p, int i) { const f2v v = p[i]; return make_float2(v.x, v.y); }
__device__ __forceinline__ void gst(gf2 *p, int i, float2 v) { f2v t; t.x = v.x; t.y = v.y; p[i] = t; }
// LDS views (address space 3)
typedef __attribute__((address_space(3))) const f2v lcf2;
__device__ __forceinline__ float2 ld2(gcf2 *p, int i) { return gld(p, i); }
__device__ __forceinline__ float2 ld2(lcf2 *p, int i) { const f2v v = p[i]; return make_float2(v.x, v.y); }

// ------------------------------------------------------------------ wave64 reductions via DPP
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_QUAD_XOR1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_MIRROR = 0x140;

// every lane ends with its 16-lane row sum; the four row sums are read with v_readlane
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += dpp_u<DPP_QUAD_XOR1>(v);
    v += dpp_u<DPP_QUAD_XOR2>(v);
    v += dpp_u<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_u<DPP_ROW_MIRROR>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    return ((uint64_t)dpp_u<CTRL>((uint32_t)(v >> 32)) << 32) | dpp_u<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    v += dpp_u64<DPP_QUAD_XOR1>(v);
    v += dpp_u64<DPP_QUAD_XOR2>(v);
    v += dpp_u64<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_u64<DPP_ROW_MIRROR>(v);
    uint64_t t = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 16 * r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 16 * r);
        t += ((uint64_t)hi << 32) | lo;
    }
    return t;
}

// ------------------------------------------------------------------ atan2 for the CFO estimates
// atan2f (OFDM.c:798, 821) as the device library's (OCML) atan2f computes it for FINITE arguments, without its
// frexp / ldexp scaling of the quotient and its inf / NaN paths: min(|x|,|y|) * rcp(max) is the library's scaled
// quotient bit for bit for normal arguments (rcp of a power-of-two-scaled mantissa scales exactly), followed by
// the same minimax polynomial and quadrant fix-ups -- the same result bit for bit wherever it is a normal float
// (when |y / x| < 2^-126 the subnormal quotient may round one subnormal step apart).  Arguments whose larger
// magnitude lies outside [2^-64, 2^64] (subnormals included) are first scaled by 2^64 or 2^-64 (exact), so rcp
// never sees a subnormal (rcp = inf, and 0 * inf would be a NaN phase) nor returns one (flushed: atan2(m, m) = 0
// instead of pi/4 for m > 2^126).  Signed zeros as atan2f: (+-0, +0) -> +-0,
// (+-0, -0) -> +-pi, (y, +-0) -> +-pi/2.  Infinite or NaN arguments are outside the contract (a CFO correlation
// sum is finite).  tests/device/atan2_check.hip compares it with atan2f on the GPU (tests/test_gpu_device.py).
__device__ __forceinline__ float atan2_cfo(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y);
    const float m = fmaxf(ax, ay);
    // the rescale sits behind a wave-uniform branch: a CFO sum is in range on every lane (it added ~6
    // VALU per call on the frame path when done unconditionally)
    if (__builtin_expect(__ballot(!(m >= 0x1p-64f && m <= 0x1p64f)) != 0ull, 0)) {
        const float sc = m < 0x1p-64f ? 0x1p64f : m > 0x1p64f ? 0x1p-64f : 1.0f;    // exact power-of-two scaling
        ax *= sc;
        ay *= sc;
    }
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    float a = mn * __builtin_amdgcn_rcpf(mx);
    a = mn > 0.f ? a : 0.f;                                        // 0 / 0 and 0 / m: 0
    const float s = a * a;
    float t = fmaf(s, __uint_as_float(0x3b2d2a58u), __uint_as_float(0xbc7a590cu));
    t = fmaf(s, t, __uint_as_float(0x3d29fb3fu));
    t = fmaf(s, t, __uint_as_float(0xbd97d4d7u));
    t = fmaf(s, t, __uint_as_float(0x3dd931b2u));
    t = fmaf(s, t, __uint_as_float(0xbe1160e6u));
    t = fmaf(s, t, __uint_as_float(0x3e4cb8bfu));
    t = fmaf(s, t, __uint_as_float(0xbeaaaa62u));
    float r = fmaf(a, s * t, a);                                   // atan(a), a in [0, 1]
    r = ay > ax ? __uint_as_float(0x3fc90fdbu) - r : r;           // pi / 2 - atan(1 / a)
    r = __builtin_signbit(x) ? __uint_as_float(0x40490fdbu) - r : r;   // pi - ... (x = -0 included)
    return copysignf(r, y);
}

__host__ __device__ constexpr int digit_rev4(int k) {
    return ((k & 3) << 4) | (k & 12) | ((k >> 4) & 3);
}

template <bool INV>
__device__ __forceinline__ void fft64(float2 (&x)[64]) { dif4<INV, 64, 0>(x); }

// ------------------------------------------------------------------ 802.11a subcarrier plan
// fftshifted bin of data subcarrier m (OFDM.c:528-547 Tx, 1063-1068 Rx)
__host__ __device__ constexpr int data_bin(int m) {
    return m < 5 ? 6 + m : m < 18 ? 7 + m : m < 24 ? 8 + m : m < 30 ? 9 + m : m < 43 ? 10 + m : 11 + m;
}
// inverse: data subcarrier index of an fftshifted bin, -1 for pilots / nulls / DC
__host__ __device__ constexpr int data_index(int bin) {
    return (bin >= 6 && bin <= 10) ? bin - 6 : (bin >= 12 && bin <= 24) ? bin - 7 : (bin >= 26 && bin <= 31) ? bin - 8
         : (bin >= 33 && bin <= 38) ? bin - 9 : (bin >= 40 && bin <= 52) ? bin - 10 : (bin >= 54 && bin <= 58) ? bin - 11 : -1;
}
// pilots {1,1,1,-1} at bins 11,25,39,53 (OFDM.c:523,531-544)
__host__ __device__ constexpr float pilot_at(int bin) {
    return bin == 11 || bin == 25 || bin == 39 ? 1.0f : (bin == 53 ? -1.0f : 0.0f);
}
// long training tones L_k at bins 6..58 (OFDM.c:494) -- sign on the data bins (all +-1)
__host__ __device__ constexpr int ltf_sign(int bin) {
    constexpr int8_t L[53] = {1, 1, -1, -1, 1, 1, -1, 1, -1, 1, 1, 1, 1, 1, 1, -1, -1, 1, 1, -1, 1, -1, 1, 1,
                              1, 1, 0, 1, -1, -1, 1, 1, -1, 1, -1, 1, -1, -1, -1, -1, -1, 1, 1, -1, -1, 1,
                              -1, 1, -1, 1, 1, 1, 1};
    return (bin >= 6 && bin <= 58) ? L[bin - 6] : 0;
}

constexpr float INV_SQRT2 = 0.70710678118654752440f;

// bit b (0..95) of a symbol's 3 MSB-first words
__device__ __forceinline__ uint32_t bit_of(const uint32_t w[3], int b) {
    return (w[b >> 5] >> (31 - (b & 31))) & 1u;
}

}  // namespace ofdm
