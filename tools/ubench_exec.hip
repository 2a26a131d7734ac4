// VALU issue microbenchmark, second pass: (1) EXEC-masked streams (does a wave64 instruction with
// one 32-lane half inactive issue faster on gfx950?), (2) 3-source ops by operand pattern
// (distinct VGPRs vs one VGPR read twice, as in a square x*x + acc), (3) per-wave issue rate at
// 1..4 waves/SIMD with 64 instructions per loop trip so branch overhead does not dominate.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_exec.hip -o tools/ubench_exec
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define ITERS 2048
#define CH 16
#define UNR 4

__device__ __forceinline__ bool active(int mode, int lane) {
    switch (mode) {
        case 0: return true;
        case 1: return lane < 32;
        default: return lane % 3 != 0;
    }
}

// OP 0 v_add_f32 a,a,k   1 v_fma a,a,b,c (distinct)   2 v_fma a,a,k,k   3 v_fma acc,x,x,acc (square)
//    4 v_bitop3 a,a,b,c   5 v_mad_u64_u32   6 v_sin_f32   7 v_fmac a,b,c
template <int OP>
__device__ __forceinline__ void op(uint32_t &x, uint32_t &y, uint32_t k, uint32_t b, uint32_t d) {
    if constexpr (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (OP == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(d));
    else if constexpr (OP == 2) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
    else if constexpr (OP == 3) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(x) : "v"(y));
    else if constexpr (OP == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(d));
    else if constexpr (OP == 5) {
        uint64_t r;
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(r) : "v"(x), "v"(b) : "s40", "s41");
        x = (uint32_t)(r >> 32);
    } else if constexpr (OP == 6) asm volatile("v_sin_f32 %0, %0" : "+v"(x));
    else if constexpr (OP == 7) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x) : "v"(b), "v"(d));
    else {   // packed f32 on register pairs (x, y)
        uint64_t xy = ((uint64_t)y << 32) | x, bd = ((uint64_t)d << 32) | b;
        if constexpr (OP == 8) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(xy) : "v"(bd));
        else if constexpr (OP == 9) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(xy) : "v"(bd));
        else asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(xy) : "v"(bd));
        x = (uint32_t)xy; y = (uint32_t)(xy >> 32);
    }
}

template <int OP>
__global__ __launch_bounds__(256) void bench(uint32_t *out, unsigned long long *cyc, uint32_t k, int mode) {
    uint32_t v[CH], w[CH];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < CH; ++c) { v[c] = threadIdx.x * 7 + c; w[c] = threadIdx.x * 5 + c; }
    uint32_t b = k + 1, d = k + 2;
    asm volatile("" : "+v"(b), "+v"(d));
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (active(mode, lane)) {
        for (int i = 0; i < ITERS; ++i) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
#pragma unroll
                for (int c = 0; c < CH; ++c) op<OP>(v[c], w[c], k, b, d);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s ^= v[c] ^ w[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[gridDim.x * 4] = r1 - r0;
}

static const char *OPN[] = {"v_add_f32", "v_fma distinct", "v_fma a,a,k,k", "v_fma x*x+acc", "v_bitop3 dist",
                            "v_mad_u64_u32", "v_sin_f32", "v_fmac a,b,c", "v_pk_add_f32", "v_pk_mul_f32",
                            "v_pk_fma_f32"};
static const char *MODEN[] = {"all 64", "lanes 0-31", "lane%3!=0"};

template <int OP>
void run(int cus, int wps, int mode, uint32_t *d_out, unsigned long long *d_cyc) {
    // whole-grid throughput: wave-instructions / (event time x shader clock x SIMDs); the clock comes
    // from s_memtime / s_memrealtime (100 MHz) of block 0 in the same launch
    const int blocks = cus * wps;   // 256 threads = 4 waves = one per SIMD per block
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 3u, mode);   // warm
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 3u, mode);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * 4 + 1);
    (void)hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost);
    const double mhz = 100.0 * (double)c[0] / (double)c[blocks * 4];
    const double instr = (double)blocks * 4 * ITERS * UNR * CH;           // wave-instructions
    const double simd_cycles = ms * 1e-3 * mhz * 1e6 * cus * 4;
    std::sort(c.begin(), c.end() - 1);
    const double med = (double)c[c.size() / 2];
    printf("%-16s %-11s waves/SIMD %d: grid %6.2f  per-wave %6.2f SIMD cycles per wave-instruction (%.0f MHz)\n",
           OPN[OP], MODEN[mode], wps, simd_cycles / instr, med / ((double)ITERS * UNR * CH), mhz);
}

template <int OP>
void sweep(int cus, uint32_t *o, unsigned long long *c) {
    for (int w = 1; w <= 4; ++w) run<OP>(cus, w, 0, o, c);

}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t *d_out;
    unsigned long long *d_cyc;
    (void)hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4);
    (void)hipMalloc(&d_cyc, (size_t)cus * 8 * 4 * 8 + 64);
    sweep<0>(cus, d_out, d_cyc);
    sweep<1>(cus, d_out, d_cyc);
    sweep<3>(cus, d_out, d_cyc);
    sweep<4>(cus, d_out, d_cyc);
    sweep<5>(cus, d_out, d_cyc);
    sweep<6>(cus, d_out, d_cyc);
    sweep<7>(cus, d_out, d_cyc);
    sweep<8>(cus, d_out, d_cyc);
    sweep<10>(cus, d_out, d_cyc);
    return 0;
}
