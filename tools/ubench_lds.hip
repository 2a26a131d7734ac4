// LDS bank-conflict attribution for frame_sync_kernel: each kernel below issues ONE of the
// sync kernel's LDS access patterns (the instruction and per-lane addresses of the gfx950 assembly of
// frame_sync_kernel<2, 3008>), ITERS times per wave, so that a rocprofv3 --pmc pass of SQ_LDS_BANK_CONFLICT and
// SQ_LDS_IDX_ACTIVE per dispatch gives its conflict and array cycles per wave-instruction.  tools/lds_attrib.py
// multiplies them by the instructions per item of each pattern (static counts from the assembly and the item's
// control flow) and compares the sum with the kernel's measured counters.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
#define ITERS 4096
#define BLOCKS 1024
#define THREADS 256

// dword index of this lane's access for iteration it (pattern-specific)
enum Pat {
    DET_RE = 0,      // detection, real parts: lane start 31 l (round 0 chunk), ds_read2_b32 (k, k + 1)
    DET_IM,          // detection, imaginary table: (im0 + 31 l) mod 980, im0 varying per iteration
    DET_R1,          // detection round 1: 15 l + floor(17 l / 64)
    MF_RE,           // matched filter, real window: lane stride 10 dwords, ds_read2_b32 (0, 1)
    MF_IM64,         // matched filter, imaginary window, even start: stride 10, ds_read2_b64 (0, 1)
    MF_IM32,         // the same with odd start: ds_read2_b32
    BPERM_SAME,      // ds_bpermute_b32, every lane reads lane 7
    BPERM_FEW,       // 61 lanes read lane 7, three lanes others
    WR128,           // capture store: ds_write_b128 at 4 l dwords (contiguous 16 B per lane)
    WR64_FR,         // matched-filter output: ds_write_b64 at lane stride 10 dwords
    RD64_FR,         // CFO / hand-off loads of fr[]: contiguous float2 per lane, ds_read_b64
    // bursts: 16 reads in flight before one s_waitcnt, as the compiler issues detection's register-block loads
    BURST_RE,        // 16 ds_read2_b32 off the real base (31 l), offsets 0..31
    BURST_REIM,      // 8 + 8 interleaved: real base 31 l, imaginary base (im0 + 31 l) mod 980
    BURST_RE_ODD,    // BURST_RE from an odd dword base
    BURST_REIM_ODD,  // BURST_REIM, real base odd
    BURST_MF,        // 16 ds_read2_b32 off a base with lane stride 10 (the matched-filter windows)
    NPAT
};

__global__ __launch_bounds__(THREADS) void lds_kernel(int pat, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) float lds[12288];          // 48 KB
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 12288; i += THREADS) lds[i] = (float)i;
    __syncthreads();
    float acc = 0.f;
    const int wbase = wv * 3072;                                         // per-wave 12 KB region
    for (int it = 0; it < ITERS; ++it) {
        int a;
        switch (pat) {
            case DET_RE: a = wbase + 31 * lane + 2 * (it & 15); break;
            case DET_IM: a = (int)((((unsigned)it * 397u) % 980u + 31u * lane) % 980u); break;
            case DET_R1: a = wbase + 15 * lane + ((17 * lane) >> 6) + 2 * (it & 7); break;
            case MF_RE: case MF_IM32: a = wbase + 10 * lane + 1 + 2 * (it & 15); break;
            case MF_IM64: a = wbase + 10 * lane + 2 * (it & 15); break;
            case WR128: a = wbase + 4 * lane; break;
            case WR64_FR: a = wbase + 10 * lane + 2 * (it & 7); break;
            default: a = wbase + 2 * lane + 2 * (it & 7); break;
        }
        const unsigned ba = (unsigned)a * 4u;
        if (pat >= BURST_RE) {
            const int odd = (pat == BURST_RE_ODD || pat == BURST_REIM_ODD) ? 1 : 0;
            const unsigned br = (unsigned)(wbase + (pat == BURST_MF ? 10 : 31) * lane + odd + 4 * (it & 3)) * 4u;
            const unsigned bi = (unsigned)(12288 - 1200 + (int)((((unsigned)it * 397u) % 980u + 31u * lane) % 980u)) * 4u;
            const bool two = pat == BURST_REIM || pat == BURST_REIM_ODD;
            const unsigned b2 = two ? bi : br;
            f2v v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15;
            asm volatile(
                "ds_read2_b32 %0, %16 offset0:0 offset1:1\n ds_read2_b32 %1, %17 offset0:0 offset1:1\n"
                "ds_read2_b32 %2, %16 offset0:2 offset1:3\n ds_read2_b32 %3, %17 offset0:2 offset1:3\n"
                "ds_read2_b32 %4, %16 offset0:4 offset1:5\n ds_read2_b32 %5, %17 offset0:4 offset1:5\n"
                "ds_read2_b32 %6, %16 offset0:6 offset1:7\n ds_read2_b32 %7, %17 offset0:6 offset1:7\n"
                "ds_read2_b32 %8, %16 offset0:8 offset1:9\n ds_read2_b32 %9, %17 offset0:8 offset1:9\n"
                "ds_read2_b32 %10, %16 offset0:10 offset1:11\n ds_read2_b32 %11, %17 offset0:10 offset1:11\n"
                "ds_read2_b32 %12, %16 offset0:12 offset1:13\n ds_read2_b32 %13, %17 offset0:12 offset1:13\n"
                "ds_read2_b32 %14, %16 offset0:14 offset1:15\n ds_read2_b32 %15, %17 offset0:14 offset1:15\n"
                "s_waitcnt lgkmcnt(0)"
                : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6), "=v"(v7), "=v"(v8), "=v"(v9),
                  "=v"(v10), "=v"(v11), "=v"(v12), "=v"(v13), "=v"(v14), "=v"(v15)
                : "v"(br), "v"(b2));
            acc += v0.x + v1.y + v2.x + v3.y + v4.x + v5.y + v6.x + v7.y + v8.x + v9.y + v10.x + v11.y + v12.x + v13.y +
                   v14.x + v15.y;
            continue;
        }
        if (pat == DET_RE || pat == DET_IM || pat == DET_R1 || pat == MF_RE || pat == MF_IM32) {
            f2v v;
            asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ba));
            acc += v.x;
        } else if (pat == MF_IM64) {
            f4v v;
            asm volatile("ds_read2_b64 %0, %1 offset0:0 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ba));
            acc += v.x + v.w;
        } else if (pat == BPERM_SAME || pat == BPERM_FEW) {
            const int src = pat == BPERM_SAME ? 7 : (lane == 5 ? 40 : lane == 33 ? 63 : lane == 60 ? 2 : 7);
            int r;
            asm volatile("ds_bpermute_b32 %0, %1, %2\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(src * 4), "v"(it + lane));
            acc += (float)r;
        } else if (pat == WR128) {
            const f4v v = {acc, 1.f, 2.f, 3.f};
            asm volatile("ds_write_b128 %0, %1\n s_waitcnt lgkmcnt(0)" :: "v"(ba), "v"(v) : "memory");
        } else if (pat == WR64_FR) {
            const f2v v = {acc, 1.f};
            asm volatile("ds_write_b64 %0, %1\n s_waitcnt lgkmcnt(0)" :: "v"(ba), "v"(v) : "memory");
        } else {
            f2v v;
            asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ba));
            acc += v.x;
        }
    }
    if (acc == 12345.f) out[blockIdx.x] = 1u;
}

int main() {
    uint32_t *out;
    if (hipMalloc(&out, BLOCKS * 4) != hipSuccess) return 1;
    static const char *names[NPAT] = {"det_re", "det_im", "det_r1", "mf_re", "mf_im64", "mf_im32", "bperm_same",
                                      "bperm_few", "wr128", "wr64_fr", "rd64_fr", "burst_re", "burst_reim",
                                      "burst_re_odd", "burst_reim_odd", "burst_mf"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // dispatch order = pattern order (tools/lds_attrib.py reads the PMC rows in this order); each pattern twice,
    // the first launch a warm-up
    for (int p = 0; p < NPAT; ++p)
        for (int r = 0; r < 2; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(lds_kernel, dim3(BLOCKS), dim3(THREADS), 0, 0, p, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            if (r) printf("%-10s %8.3f ms  %.2f ns per wave-instruction per CU\n", names[p], ms,
                          ms * 1e6 / ((double)BLOCKS * (THREADS / 64) * ITERS / 256));
        }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
