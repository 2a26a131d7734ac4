// frame_sync_kernel's LDS reads replayed with the kernel's own LDS layout and per-item geometry:
// block layout [acc 64 dwords | imaginary table 1108 | 4 wave regions of 3020 dwords], capture start rx_start drawn
// per item, off = rx_start & 3, im0 = rx_start mod 980.  Each pattern runs ITEMS items per wave; a rocprofv3 --pmc
// pass of SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS per dispatch prices it per instruction.
//   0 det0   round-0 detection: lane l's real block at rbase + off + 31 l, imaginary at (im0 + 31 l) mod 980, the
//            80 + 80 ds_read2_b32 (offsets k, k + 1) of blocks 0..4
//   1 det0_re  the same, real parts only          2 det0_im  imaginary parts only
//   3 mf     matched-filter windows: lane u's run start s0(u) (coarse window, LTF pair, data symbols, MF_RUN 5),
//            29 floats real + 29 imaginary from n_lo = p + 2 s0 - 20 as 14 ds_read2_b32 + 1 ds_read_b32 each
//   4 mf_re  real windows only                    5 mf_im  imaginary windows only
//   6 mf_im_nowrap  imaginary windows read at imt + im0 + n_lo without the period wrap
//   7 mf_re_even    real windows with the lane starts rounded down to even dwords (aligned pairs)
//   8 s10      one set, lane stride 10 dwords (29-float windows)       9 s10_b64  the same, even starts, ds_read_b64
//  10 s32      lane stride 32 dwords (sanity: every lane on one bank)  11 mf_b64   the MF sets, even starts, ds_read_b64
//  12 det1_re  round-1 detection real parts: B1 + 15 l + floor(17 l / 64), 4 blocks
//  13 s31      lane stride 31 (round-0 real parts), 29-float windows   14 s10_0 lane stride 10 at a fixed base (no it term)
//  15 det0_u64  round-0 detection (real + imaginary) as ds_read_b64 at 4-byte-aligned (unaligned) addresses
//  16 mf_u64    matched-filter windows (real + imaginary) as ds_read_b64 at their own (unaligned) starts
//  (15, 16 also check the loaded values: out[] counts lanes whose unaligned 8-byte reads returned wrong data)
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_item.hip -o tools/ubench_lds_item
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f2v __attribute__((ext_vector_type(2)));
#define ITEMS 256
#define BLOCKS 768
#define THREADS 256
#define NPAT 17

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float read_pairs8(uint32_t a, float acc) {   // 8 pairs at dword offsets 0..15 from a
    f2v v0, v1, v2, v3, v4, v5, v6, v7;
    asm volatile("ds_read2_b32 %0, %8 offset0:0 offset1:1\n ds_read2_b32 %1, %8 offset0:2 offset1:3\n"
                 "ds_read2_b32 %2, %8 offset0:4 offset1:5\n ds_read2_b32 %3, %8 offset0:6 offset1:7\n"
                 "ds_read2_b32 %4, %8 offset0:8 offset1:9\n ds_read2_b32 %5, %8 offset0:10 offset1:11\n"
                 "ds_read2_b32 %6, %8 offset0:12 offset1:13\n ds_read2_b32 %7, %8 offset0:14 offset1:15\n"
                 "s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6), "=v"(v7) : "v"(a));
    return acc + v0.x + v1.y + v2.x + v3.y + v4.x + v5.y + v6.x + v7.y;
}
__device__ __forceinline__ float read_window28_b64(uint32_t a, float acc) {   // 14 ds_read_b64 from a (8-B aligned)
    f2v v0, v1, v2, v3, v4, v5, v6;
    asm volatile("ds_read_b64 %0, %7\n ds_read_b64 %1, %7 offset:8\n ds_read_b64 %2, %7 offset:16\n"
                 "ds_read_b64 %3, %7 offset:24\n ds_read_b64 %4, %7 offset:32\n ds_read_b64 %5, %7 offset:40\n"
                 "ds_read_b64 %6, %7 offset:48\n s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6) : "v"(a));
    acc += v0.x + v1.y + v2.x + v3.y + v4.x + v5.y + v6.x;
    asm volatile("ds_read_b64 %0, %7 offset:56\n ds_read_b64 %1, %7 offset:64\n ds_read_b64 %2, %7 offset:72\n"
                 "ds_read_b64 %3, %7 offset:80\n ds_read_b64 %4, %7 offset:88\n ds_read_b64 %5, %7 offset:96\n"
                 "ds_read_b64 %6, %7 offset:104\n s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6) : "v"(a));
    return acc + v0.x + v1.y + v2.x + v3.y + v4.x + v5.y + v6.x;
}
// 8 ds_read_b64 at dword offsets 0, 2, .., 14 from a (any 4-byte alignment); returns the number of wrong values
// (lds[i] = i)
__device__ __forceinline__ int read_u64x8(uint32_t a, uint32_t lds0, float &acc) {
    f2v v0, v1, v2, v3, v4, v5, v6, v7;
    asm volatile("ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:8\n ds_read_b64 %2, %8 offset:16\n"
                 "ds_read_b64 %3, %8 offset:24\n ds_read_b64 %4, %8 offset:32\n ds_read_b64 %5, %8 offset:40\n"
                 "ds_read_b64 %6, %8 offset:48\n ds_read_b64 %7, %8 offset:56\n s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6), "=v"(v7) : "v"(a));
    const float b = (float)((a - lds0) / 4u);
    int bad = 0;
    const f2v vv[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
    for (int m = 0; m < 8; ++m) bad += (vv[m].x != b + 2 * m) + (vv[m].y != b + 2 * m + 1);
    acc += v0.x + v7.y;
    return bad;
}
__device__ __forceinline__ float read_window29(uint32_t a, float acc) {   // 14 pairs + 1 dword from a (bytes)
    f2v v0, v1, v2, v3, v4, v5, v6;
    float w;
    acc = read_pairs8(a, acc);
    asm volatile("ds_read2_b32 %0, %8 offset0:16 offset1:17\n ds_read2_b32 %1, %8 offset0:18 offset1:19\n"
                 "ds_read2_b32 %2, %8 offset0:20 offset1:21\n ds_read2_b32 %3, %8 offset0:22 offset1:23\n"
                 "ds_read2_b32 %4, %8 offset0:24 offset1:25\n ds_read2_b32 %5, %8 offset0:26 offset1:27\n"
                 "ds_read_b32 %7, %8 offset:112\n s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6), "=v"(w) : "v"(a));
    (void)v6;
    return acc + v0.x + v1.y + v2.x + v3.y + v4.x + v5.y + w;
}

// matched-filter run start s0 of lane u (ofdm_frame.hip: 7 runs over [80, 112), 26 over [192, 320), 13 per data symbol)
__device__ __forceinline__ int mf_s0(int u) {
    if (u < 7) return 80 + 5 * u;
    if (u < 33) return 192 + 5 * (u - 7);
    const int d = (u - 33) / 13, k = u - 33 - 13 * d;
    return 336 + 80 * d + 5 * k;
}

__global__ __launch_bounds__(THREADS) void item_kernel(int pat, uint32_t *out) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 64 + 1108 + 4 * 3020; i += THREADS) lds[i] = (float)i;
    __syncthreads();
    float acc = 0.f;
    int bad = 0;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float *)lds;
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t h = hash32((uint32_t)(blockIdx.x * 4 + wv) * 7919u + (uint32_t)it);
        const int rx_start = (int)(h % 6792u), off = rx_start & 3, im0 = rx_start % 980;
        const int rbase = 1172 + 3020 * wv + off;
        if (pat <= 2) {
            const uint32_t ar = lds0 + 4u * (uint32_t)(rbase + 31 * lane);
            const uint32_t ai = lds0 + 4u * (uint32_t)(64 + (im0 + 31 * lane) % 980);
            for (int b = 0; b < 5; ++b) {                 // blocks 0..4 of 16 samples
                if (pat != 2) acc = read_pairs8(ar + 64u * b, acc);
                if (pat != 1) acc = read_pairs8(ai + 64u * b, acc);
            }
        } else if (pat == 15) {
            const uint32_t ar = lds0 + 4u * (uint32_t)(rbase + 31 * lane);
            const uint32_t ai = lds0 + 4u * (uint32_t)(64 + (im0 + 31 * lane) % 980);
            for (int b = 0; b < 5; ++b) {
                bad += read_u64x8(ar + 64u * b, lds0, acc);
                bad += read_u64x8(ai + 64u * b, lds0, acc);
            }
        } else if (pat == 16) {
            if (lane < 59) {
                const int p = 11 + (int)((h >> 8) % 1900u);
                const int n_lo = p + 2 * mf_s0(lane) - 20;
                bad += read_u64x8(lds0 + 4u * (uint32_t)(rbase + n_lo), lds0, acc);
                bad += read_u64x8(lds0 + 4u * (uint32_t)(rbase + n_lo) + 64u, lds0, acc);
                bad += read_u64x8(lds0 + 4u * (uint32_t)(64 + (im0 + n_lo) % 980), lds0, acc);
                bad += read_u64x8(lds0 + 4u * (uint32_t)(64 + (im0 + n_lo) % 980) + 64u, lds0, acc);
            }
        } else if (pat >= 8 && pat != 11) {
            const int rb = 1172 + 3020 * wv;
            int st = pat == 8 ? rb + 10 * lane + (it & 1) : pat == 9 ? rb + 10 * lane : pat == 10 ? 32 * lane + (it & 7)
                   : pat == 12 ? rb + off + 1984 + 15 * lane + ((17 * lane) >> 6) : pat == 13 ? rb + off + 31 * lane
                   : rb + 10 * lane;
            const uint32_t a = lds0 + 4u * (uint32_t)st;
            if (pat == 9) acc = read_window28_b64(a, acc);
            else if (pat == 12) { for (int b = 0; b < 4; ++b) acc = read_pairs8(a + 64u * b, acc); }
            else acc = read_window29(a, acc);
        } else if (lane < 59) {
            const int p = 11 + (int)((h >> 8) % 1900u);
            const int n_lo = p + 2 * mf_s0(lane) - 20;
            int rr = rbase + n_lo;
            if (pat == 7) rr &= ~1;
            const int ii = pat == 6 ? 64 + im0 + n_lo : 64 + (im0 + n_lo) % 980;
            if (pat == 11) { acc = read_window28_b64(lds0 + 4u * (uint32_t)(rr & ~1), acc); continue; }
            if (pat == 3 || pat == 4 || pat == 7) acc = read_window29(lds0 + 4u * (uint32_t)rr, acc);
            if (pat == 3 || pat == 5 || pat == 6) acc = read_window29(lds0 + 4u * (uint32_t)(ii < 64 + 3000 ? ii : 64), acc);
        }
    }
    if (acc == 12345.f) out[blockIdx.x] = 1u;
    if (bad) atomicAdd(&out[BLOCKS], 1u);
}

int main() {
    uint32_t *out;
    if (hipMalloc(&out, (BLOCKS + 1) * 4) != hipSuccess) return 1;
    static const char *names[NPAT] = {"det0", "det0_re", "det0_im", "mf", "mf_re", "mf_im", "mf_im_nowrap", "mf_re_even",
                                      "s10", "s10_b64", "s32", "mf_b64", "det1_re", "s31", "s10_0", "det0_u64", "mf_u64"};
    const size_t lds = (64 + 1108 + 4 * 3020) * 4;
    for (int p = 0; p < NPAT; ++p)
        for (int r = 0; r < 2; ++r) {
            if (hipMemset(out + BLOCKS, 0, 4) != hipSuccess) return 1;
            hipLaunchKernelGGL(item_kernel, dim3(BLOCKS), dim3(THREADS), lds, 0, p, out);
            uint32_t nbad = 0;
            if (hipMemcpy(&nbad, out + BLOCKS, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (r) printf("%s done, %u blocks with wrong values\n", names[p], nbad);
        }
    return 0;
}
