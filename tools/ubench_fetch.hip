// FETCH_SIZE calibration for the access widths K3c uses: how many bytes rocprofv3's
// FETCH_SIZE reports for a known byte count read from HBM by
//   0  wide     float4 per lane, coalesced (the guide's calibrated case: FETCH_SIZE = 1/2 of the bytes)
//   1  f2       float2 per lane, coalesced (the width of K3c's group-prologue loads of Tx rows 16..79)
//   2  warm     one 4-byte global_load_lds per 128-B line (K3c's L2 warm-up of the next item's rows)
//   3  warm+f2  K3c's pattern: each block warms item i + 1 while it reads item i (64 KB and 16 KB items)
// Each kernel reads a 1 GiB buffer (4x the 256 MiB Infinity Cache) once; one launch per kernel id.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_fetch.hip -o tools/ubench_fetch
// run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o run --output-format csv -- tools/ubench_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(1) << 30;

__global__ __launch_bounds__(256) void k_wide(const float4 *p, size_t n, float *out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;        // keeps the loads alive, never true for the zero-filled buffer
}

__global__ __launch_bounds__(256) void k_f2(const float2 *p, size_t n, float *out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float2 v = p[i];
        s += v.x + v.y;
    }
    if (s == 1234.5f) out[0] = s;
}

// one lane per 128-B line, 4 bytes into a dummy LDS word (the K3c warm-up instruction)
__device__ __forceinline__ void warm_lines(const char *p, size_t lines) {
    __shared__ uint32_t dummy[64];
    for (size_t l = blockIdx.x * 256 + threadIdx.x; l < lines; l += (size_t)gridDim.x * 256)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(p + 128 * l),
                                         (__attribute__((address_space(3))) void *)dummy, 4, 0, 0);
}

__global__ __launch_bounds__(256) void k_warm(const char *p, size_t lines) { warm_lines(p, lines); }

// K3c's pattern: a block owns items of ITEM bytes (K3c: 64 rows x 1 KB of Tx samples per 64-frame group); while
// it reads item i as float2 it warms item i + 1 with one 4-byte global_load_lds per 128-B line
template <int ITEM>
__global__ __launch_bounds__(256) void k_warm_f2(const char *p, size_t bytes, float *out) {
    __shared__ uint32_t dummy[64];
    const size_t n_items = bytes / ITEM;
    float s = 0.f;
    for (size_t it = blockIdx.x; it < n_items; it += gridDim.x) {
        const size_t nx = it + gridDim.x;
        if (nx < n_items)
            for (int l = threadIdx.x; l < ITEM / 128; l += 256)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(p + nx * ITEM + 128 * l),
                                                 (__attribute__((address_space(3))) void *)dummy, 4, 0, 0);
        const float2 *q = reinterpret_cast<const float2 *>(p + it * ITEM);
        for (int i = threadIdx.x; i < ITEM / 8; i += 256) {
            const float2 v = q[i];
            s += v.x + v.y;
        }
    }
    if (s == 1234.5f) out[0] = s;
}

int main() {
    char *buf = nullptr;
    float *out = nullptr;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, BYTES);
    hipDeviceSynchronize();
    const size_t lines = BYTES / 128;
    const int grid = 256 * 8;
    hipLaunchKernelGGL(k_wide, dim3(grid), dim3(256), 0, 0, (const float4 *)buf, BYTES / 16, out);
    hipLaunchKernelGGL(k_f2, dim3(grid), dim3(256), 0, 0, (const float2 *)buf, BYTES / 8, out);
    hipLaunchKernelGGL(k_warm, dim3(grid), dim3(256), 0, 0, (const char *)buf, lines);
    // K3c's grid: 3 resident blocks per CU x 256 CUs; its item is 64 KB
    hipLaunchKernelGGL(k_warm_f2<65536>, dim3(768), dim3(256), 0, 0, (const char *)buf, BYTES, out);
    hipLaunchKernelGGL(k_warm_f2<16384>, dim3(768), dim3(256), 0, 0, (const char *)buf, BYTES, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("bytes per kernel %zu (wide, f2, warm: %zu lines x 128 B, warm+f2 64 KB / 16 KB items)\n", BYTES, lines);
    hipFree(buf);
    hipFree(out);
    return 0;
}
