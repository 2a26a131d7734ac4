// HBM copy ceiling at K1's size: 2^24 x 512 B read + the same written, as
//   copy4    float4 per lane, one 16-B load + store per lane per 1-KB wave chunk, grid of one chunk per wave
//   copy4nt  the same with non-temporal stores
//   copy4gs  grid-stride loop over the chunks (2048 blocks of 256 threads), 4 chunks in flight per wave
//   copyb8   K1's batch shape without the transform: a wave loads 8 KB (8 x 16 B per lane, all in flight), then
//            stores it (nt)
//   copydma8 the same through LDS as K1 moves it: 8 LDS-DMA loads of 1 KB (nt), s_waitcnt, ds_read_b128, nt
//            stores; 32 KB of LDS per 256-thread block (5 blocks per CU, as K1)
//   copybN   the copyb8 shape with N KB per wave (N = 2, 4)
//   copyb8w1 copyb8 in one-wave blocks
//   copypipe persistent waves (4 per SIMD), each streaming 8-KB batches with the next batch's loads issued before
//            the current batch's stores
//   dmapipe  the same through LDS: two 8-KB LDS-DMA buffers per wave, batch k+1 loading while batch k is stored
//   dma8bN   copydma8 held to N blocks (4 N waves) per CU by dynamic LDS padding (N = 2, 3, 4)
//   b8bN     copyb8 held to N blocks per CU the same way (N = 2, 3, 4, 6)
// Prints GB/s (read + written bytes / time) per variant, best of 5 launches.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_copy.hip -o tools/ubench_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void copy4(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) {
        const f4v v = in[i];
        if (NT) __builtin_nontemporal_store(v, out + i); else out[i] = v;
    }
}

__global__ __launch_bounds__(256) void copy4gs(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256 * 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 * 4 + threadIdx.x; i < n4; i += stride) {
        f4v v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + 256 * u < n4 ? in[i + 256 * u] : f4v{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i + 256 * u < n4) __builtin_nontemporal_store(v[u], out + i + 256 * u);
    }
}

__global__ __launch_bounds__(256) void copyb8(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 512 + (threadIdx.x & 63);
    f4v v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base + 64 * u < n4 ? __builtin_nontemporal_load(in + base + 64 * u) : f4v{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 8; ++u) if (base + 64 * u < n4) __builtin_nontemporal_store(v[u], out + base + 64 * u);
}

__global__ __launch_bounds__(256) void copydma8(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    __shared__ __attribute__((aligned(16))) f4v buf[4][512];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t base = ((int64_t)blockIdx.x * 4 + wv) * 512;
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (base + 64 * u + lane < n4)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(in + base + 64 * u + lane),
                                             (__attribute__((address_space(3))) void *)(&buf[wv][64 * u]), 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    typedef __attribute__((address_space(3))) const f4v lf4;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const f4v v = *(lf4 *)&buf[wv][64 * u + lane];
        if (base + 64 * u + lane < n4) __builtin_nontemporal_store(v, out + base + 64 * u + lane);
    }
}

template <int N>
__global__ __launch_bounds__(256) void copybn(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * N + (threadIdx.x & 63);
    f4v v[N];
#pragma unroll
    for (int u = 0; u < N; ++u) v[u] = base + 64 * u < n4 ? __builtin_nontemporal_load(in + base + 64 * u) : f4v{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < N; ++u) if (base + 64 * u < n4) __builtin_nontemporal_store(v[u], out + base + 64 * u);
}

__global__ __launch_bounds__(64) void copyb8w1(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int64_t base = (int64_t)blockIdx.x * 512 + threadIdx.x;
    f4v v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base + 64 * u < n4 ? __builtin_nontemporal_load(in + base + 64 * u) : f4v{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 8; ++u) if (base + 64 * u < n4) __builtin_nontemporal_store(v[u], out + base + 64 * u);
}

__global__ __launch_bounds__(256) void copypipe(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    const int lane = threadIdx.x & 63;
    const int64_t nb = n4 / 512, nw = (int64_t)gridDim.x * 4;
    int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    f4v v[8], w[8];
    if (b < nb) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(in + b * 512 + 64 * u + lane);
    }
    for (; b < nb; b += nw) {
        const int64_t bn = b + nw;
        if (bn < nb) {
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = __builtin_nontemporal_load(in + bn * 512 + 64 * u + lane);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) __builtin_nontemporal_store(v[u], out + b * 512 + 64 * u + lane);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = w[u];
    }
}

__global__ __launch_bounds__(256) void dmapipe(const f4v *__restrict__ in, f4v *__restrict__ out, int64_t n4) {
    __shared__ __attribute__((aligned(16))) f4v buf[4][2][512];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nb = n4 / 512, nw = (int64_t)gridDim.x * 4;
    int64_t b = (int64_t)blockIdx.x * 4 + wv;
    auto issue = [&](int64_t bb, int k) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(in + bb * 512 + 64 * u + lane),
                                             (__attribute__((address_space(3))) void *)(&buf[wv][k][64 * u]), 16, 0, 2);
    };
    if (b < nb) issue(b, 0);
    typedef __attribute__((address_space(3))) const f4v lf4;
    for (int k = 0; b < nb; b += nw, k ^= 1) {
        const int64_t bn = b + nw;
        if (bn < nb) {
            issue(bn, k ^ 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // batch b landed (in-order counter), bn in flight
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const f4v v = *(lf4 *)&buf[wv][k][64 * u + lane];
            __builtin_nontemporal_store(v, out + b * 512 + 64 * u + lane);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // LDS reads of buffer k done before it is refilled
    }
}

int main() {
    const int64_t n4 = (int64_t)1 << 29;                   // 2^24 transforms x 32 chunks of 16 B = 8 GiB
    f4v *a, *b;
    if (hipMalloc(&a, n4 * 16) != hipSuccess || hipMalloc(&b, n4 * 16) != hipSuccess) return 1;
    if (hipMemset(a, 0, n4 * 16) != hipSuccess || hipMemset(b, 0, n4 * 16) != hipSuccess) return 1;
    if (hipFuncSetAttribute((const void *)copydma8, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024) != hipSuccess ||
        hipFuncSetAttribute((const void *)copyb8, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024) != hipSuccess)
        printf("hipFuncSetAttribute failed\n");
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    const char *names[17] = {"copy4", "copy4nt", "copy4gs", "copyb8", "copydma8", "copyb2", "copyb4", "copyb8w1",
                             "copypipe", "dmapipe", "dma8b2", "dma8b3", "dma8b4", "b8b2", "b8b3", "b8b4", "b8b6"};
    const int nblk[17] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 4, 2, 3, 4, 6};
    for (int v = 0; v < 17; ++v) {
        const size_t pad = nblk[v] ? 160 * 1024 / nblk[v] - (v < 13 ? 32 * 1024 : 0) - 1024 : 0;
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            if (hipEventRecord(e0) != hipSuccess) return 1;
            if (v == 0) hipLaunchKernelGGL(copy4<false>, dim3((unsigned)(n4 / 256)), dim3(256), 0, 0, a, b, n4);
            else if (v == 1) hipLaunchKernelGGL(copy4<true>, dim3((unsigned)(n4 / 256)), dim3(256), 0, 0, a, b, n4);
            else if (v == 2) hipLaunchKernelGGL(copy4gs, dim3(2048), dim3(256), 0, 0, a, b, n4);
            else if (v == 3) hipLaunchKernelGGL(copyb8, dim3((unsigned)(n4 / 2048)), dim3(256), 0, 0, a, b, n4);
            else if (v == 4) hipLaunchKernelGGL(copydma8, dim3((unsigned)(n4 / 2048)), dim3(256), 0, 0, a, b, n4);
            else if (v == 5) hipLaunchKernelGGL(copybn<2>, dim3((unsigned)(n4 / 512)), dim3(256), 0, 0, a, b, n4);
            else if (v == 6) hipLaunchKernelGGL(copybn<4>, dim3((unsigned)(n4 / 1024)), dim3(256), 0, 0, a, b, n4);
            else if (v == 7) hipLaunchKernelGGL(copyb8w1, dim3((unsigned)(n4 / 512)), dim3(64), 0, 0, a, b, n4);
            else if (v == 8) hipLaunchKernelGGL(copypipe, dim3(1024), dim3(256), 0, 0, a, b, n4);
            else if (v == 9) hipLaunchKernelGGL(dmapipe, dim3(512), dim3(256), 0, 0, a, b, n4);
            else if (v < 13) hipLaunchKernelGGL(copydma8, dim3((unsigned)(n4 / 2048)), dim3(256), pad, 0, a, b, n4);
            else hipLaunchKernelGGL(copyb8, dim3((unsigned)(n4 / 2048)), dim3(256), pad, 0, a, b, n4);
            if (hipGetLastError() != hipSuccess) { printf("%s: launch failed\n", names[v]); break; }
            if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
            if (ms < best) best = ms;
        }
        printf("%-8s %.3f ms  %.0f GB/s (read + written)\n", names[v], best, 2.0 * n4 * 16 / (best * 1e-3) / 1e9);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
