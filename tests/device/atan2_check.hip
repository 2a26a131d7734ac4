// atan2_check.hip -- test program (tests/test_gpu_device.py): the frame kernel's atan2_cfo (ofdm_device.h) against
// the device library's atan2f on the same arguments, on the GPU.
// usage: atan2_check IN OUT    IN: n pairs (y, x) float32; OUT: n pairs (atan2_cfo, atan2f) float32
#include <cstdio>
#include <vector>
#include "ofdm_device.h"

__global__ void atan2_kernel(const float2 *yx, float2 *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float2(ofdm::atan2_cfo(yx[i].x, yx[i].y), atan2f(yx[i].x, yx[i].y));
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: atan2_check IN OUT\n"); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    std::vector<float2> h;
    float2 v;
    while (fread(&v, sizeof v, 1, f) == 1) h.push_back(v);
    fclose(f);
    const int n = (int)h.size();
    if (n == 0 || n > (1 << 24)) { fprintf(stderr, "bad input size %d\n", n); return 2; }
    float2 *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc(&d_in, n * sizeof(float2)) != hipSuccess || hipMalloc(&d_out, n * sizeof(float2)) != hipSuccess) return 3;
    if (hipMemcpy(d_in, h.data(), n * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) return 3;
    hipLaunchKernelGGL(atan2_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, (const float2 *)d_in, d_out, n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 3;
    if (hipMemcpy(h.data(), d_out, n * sizeof(float2), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    hipFree(d_in);
    hipFree(d_out);
    FILE *o = fopen(argv[2], "wb");
    if (!o || fwrite(h.data(), sizeof(float2), n, o) != (size_t)n) { perror(argv[2]); return 2; }
    fclose(o);
    return 0;
}
