// VALU issue-cost microbenchmark for the instructions the Rx loop is built from (Philox multiply,
// Box-Muller transcendentals, DPP moves, FFT fma/add).  8 independent chains per lane, so the
// numbers are throughput, not latency.  Cycles from s_memtime around the loop (per wave); reported
// as SIMD cycles per wave-instruction at k waves/SIMD = cycles / (k * instructions).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <utility>

#define ITERS 512
#define CH 8

template <int OP>
__device__ __forceinline__ void step(uint32_t (&v)[CH], uint32_t k) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        uint32_t x = v[c];
        if constexpr (OP == 0) {          // v_fma_f32
            asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 1) {   // v_add_u32
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 2) {   // v_mad_u64_u32
            uint64_t r;
            asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(r) : "v"(x), "v"(k) : "s40", "s41");
            x = (uint32_t)r;
        } else if constexpr (OP == 3) {   // v_mul_lo_u32
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 4) {   // v_mul_hi_u32
            asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 5) {   // v_mul_u32_u24
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 6) {   // v_mul_hi_u32_u24
            asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 7) {   // v_bitop3_b32
            asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 8) {   // v_log_f32
            asm volatile("v_log_f32 %0, %0" : "+v"(x));
        } else if constexpr (OP == 9) {   // v_sin_f32
            asm volatile("v_sin_f32 %0, %0" : "+v"(x));
        } else if constexpr (OP == 10) {  // v_sqrt_f32
            asm volatile("v_sqrt_f32 %0, %0" : "+v"(x));
        } else if constexpr (OP == 11) {  // v_rcp_f32
            asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
        } else if constexpr (OP == 12) {  // v_mov_b32 dpp quad_perm
            asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
        } else if constexpr (OP == 13) {  // v_add_f32 with dpp source
            asm volatile("v_add_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 14) {  // v_cvt_f32_u32
            asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
        } else if constexpr (OP == 15) {  // v_pk_fma_f32 (2 lanes of f32 per instruction)
            uint64_t y = ((uint64_t)x << 32) | x;
            asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(y));
            x = (uint32_t)y;
        } else if constexpr (OP == 16) {  // v_mul_f32
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 17) {  // v_xor_b32
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k));
        } else if constexpr (OP == 18) {  // v_mov_b32 dpp row_mirror
            asm volatile("v_mov_b32_dpp %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x));
        } else if constexpr (OP == 19) {  // v_exp_f32
            asm volatile("v_exp_f32 %0, %0" : "+v"(x));
        }
        v[c] = x;
    }
}

template <int OP>
__global__ __launch_bounds__(256) void bench(uint32_t *out, unsigned long long *cyc, uint32_t k) {
    uint32_t v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 7 + c;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) step<OP>(v, k);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}

static const char *NAMES[] = {"v_fma_f32", "v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
                              "v_mul_u32_u24", "v_mul_hi_u32_u24", "v_bitop3_b32", "v_log_f32", "v_sin_f32",
                              "v_sqrt_f32", "v_rcp_f32", "v_mov_dpp_quad", "v_add_f32_dpp", "v_cvt_f32_u32",
                              "v_pk_fma_f32", "v_mul_f32", "v_xor_b32", "v_mov_dpp_rowmirror", "v_exp_f32"};

template <int OP>
void run(int cus, int wps, uint32_t *d_out, unsigned long long *d_cyc) {
    const int blocks = cus * wps;   // 256 threads = 4 waves = 1 per SIMD per block
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 3u);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks * 4);
    hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[c.size() / 2];
    const double n = (double)ITERS * CH;
    // s_memtime counts at the shader clock; per-SIMD cycles per wave-instruction with wps waves sharing it
    printf("%-20s waves/SIMD %d: %6.2f SIMD cycles per wave-instruction (per-wave %6.2f)\n", NAMES[OP], wps,
           med / (n * wps), med / n);
}

template <int... OPS>
void run_all(int cus, int wps, uint32_t *o, unsigned long long *c, std::integer_sequence<int, OPS...>) {
    (run<OPS>(cus, wps, o, c), ...);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("device %s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
    uint32_t *d_out;
    unsigned long long *d_cyc;
    hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&d_cyc, (size_t)cus * 8 * 4 * 8);
    for (int w : {1, 2, 4}) run_all(cus, w, d_out, d_cyc, std::make_integer_sequence<int, 20>{});
    return 0;
}
