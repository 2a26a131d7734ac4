// HBM copy ceiling at K1's size: 2^24 x 512 B read + the same written, as
//   copy4    float4 per lane, one 16-B load + store per lane per 1-KB wave chunk, grid of one chunk per wave
//   copy4nt  the same with non-temporal stores
//   copy4gs  grid-stride loop over the chunks (2048 blocks of 256 threads), 4 chunks in flight per wave
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

int main() {
    const int64_t n4 = (int64_t)1 << 29;                   // 2^24 transforms x 32 chunks of 16 B = 8 GiB
    f4v *a, *b;
    if (hipMalloc(&a, n4 * 16) != hipSuccess || hipMalloc(&b, n4 * 16) != hipSuccess) return 1;
    if (hipMemset(a, 0, n4 * 16) != hipSuccess || hipMemset(b, 0, n4 * 16) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    const char *names[3] = {"copy4", "copy4nt", "copy4gs"};
    for (int v = 0; v < 3; ++v) {
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            if (hipEventRecord(e0) != hipSuccess) return 1;
            if (v == 0) hipLaunchKernelGGL(copy4<false>, dim3((unsigned)(n4 / 256)), dim3(256), 0, 0, a, b, n4);
            else if (v == 1) hipLaunchKernelGGL(copy4<true>, dim3((unsigned)(n4 / 256)), dim3(256), 0, 0, a, b, n4);
            else hipLaunchKernelGGL(copy4gs, dim3(2048), dim3(256), 0, 0, a, b, n4);
            if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
            if (ms < best) best = ms;
        }
        printf("%-8s %.3f ms  %.0f GB/s (read + written)\n", names[v], best, 2.0 * n4 * 16 / (best * 1e-3) / 1e9);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
