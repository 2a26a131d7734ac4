// VALU issue cost vs VGPR operands (gfx950).  Each case is one asm block with hard-coded registers:
// 64 independent instructions per loop trip (destinations rotate over v40..v47, sources fixed), so
// the figure is pure issue throughput.  VGPR bank = register number mod 4.
//
// Question: is a 3-source VALU op (v_fma_f32, v_bitop3_b32) slower because it reads three VGPRs,
// or only when two of its sources share a bank?  tools/ubench_exec.hip could not tell (the
// compiler chose its registers there).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_bank.hip -o tools/ubench_bank
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define ITERS 1024
#define STR2(x) #x
#define STR(x) STR2(x)

#define R8(I) I(40) I(41) I(42) I(43) I(44) I(45) I(46) I(47)
#define R64(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I)
#define P4(I) I(40, 41) I(42, 43) I(44, 45) I(46, 47)
#define P64(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I) P4(I)

#define INIT                                                                                         \
    "v_mov_b32 v1, 1.0\n v_mov_b32 v2, 0.5\n v_mov_b32 v3, 0.25\n v_mov_b32 v4, 1.5\n"              \
    "v_mov_b32 v5, 2.0\n v_mov_b32 v6, 0.75\n v_mov_b32 v7, 3.0\n v_mov_b32 v8, 0.125\n"              \
    "v_mov_b32 v9, 1.0\n v_mov_b32 v12, 1.25\n s_mov_b32 s20, 1.0\n"
#define LOOP_HEAD "s_mov_b32 s21, " STR(ITERS) "\n 1:\n"
#define LOOP_TAIL "s_sub_u32 s21, s21, 1\n s_cmp_lg_u32 s21, 0\n s_cbranch_scc1 1b\n"
#define CLOB                                                                                          \
    "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v40", "v41", "v42",   \
        "v43", "v44", "v45", "v46", "v47", "s20", "s21", "s22", "s23", "vcc", "scc"

#define C0(D) "v_fma_f32 v" #D ", v1, v2, v3\n"          // 3 VGPRs, banks 1,2,3
#define C1(D) "v_fma_f32 v" #D ", v4, v8, v12\n"         // 3 VGPRs, all bank 0
#define C2(D) "v_fma_f32 v" #D ", v4, v8, v1\n"          // 3 VGPRs, two in bank 0
#define C3(D) "v_fma_f32 v" #D ", v1, v1, v2\n"          // src0 == src1
#define C4(D) "v_fma_f32 v" #D ", v1, v2, v2\n"          // src1 == src2
#define C5(D) "v_fma_f32 v" #D ", v1, s20, v2\n"         // 2 VGPRs + SGPR
#define C6(D) "v_add_f32 v" #D ", v1, v2\n"              // 2 VGPRs, banks 1,2
#define C7(D) "v_add_f32 v" #D ", v4, v8\n"              // 2 VGPRs, same bank
#define C8(D) "v_bitop3_b32 v" #D ", v1, v2, v3 bitop3:0x96\n"
#define C9(D) "v_bitop3_b32 v" #D ", v1, v2, s20 bitop3:0x96\n"
#define C10(D) "v_fmac_f32 v" #D ", v1, v2\n"            // dst is the 3rd source
#define C11(D) "v_mul_f32 v" #D ", v1, v2\n"
#define C12(D) "v_fmamk_f32 v" #D ", v1, 0x3f3504f3, v2\n"
#define C13(D) "v_cndmask_b32 v" #D ", v1, v2, vcc\n"
#define C14(D) "v_sin_f32 v" #D ", v1\n"
#define C15(D) "v_alignbit_b32 v" #D ", v1, v2, 31\n"
#define M64(A, B) "v_mad_u64_u32 v[" #A ":" #B "], s[22:23], v1, s20, 0\n"
#define PKF(A, B) "v_pk_fma_f32 v[" #A ":" #B "], v[2:3], v[4:5], v[6:7]\n"
#define PKA(A, B) "v_pk_add_f32 v[" #A ":" #B "], v[2:3], v[4:5]\n"

#define D0(D) "v_add_f32 v" #D ", s20, v1\n"             // VOP2, SGPR
#define D1(D) "v_add_f32 v" #D ", 1.0, v1\n"             // VOP2, inline constant
#define D2(D) "v_mul_f32 v" #D ", 0x3f3504f3, v1\n"      // VOP2, literal
#define D3(D) "v_lshlrev_b32 v" #D ", 6, v1\n"           // VOP2, inline integer
#define D4(D) "v_xor_b32 v" #D ", s20, v1\n"             // VOP2, SGPR
#define D5(D) "v_alignbit_b32 v" #D ", v1, v2, v3\n"     // VOP3, all VGPR
#define D6(D) "v_fma_f32 v" #D ", -v1, v2, v3\n"         // VOP3, neg modifier
#define D7(D) "v_mul_f32_e64 v" #D ", v1, -v2\n"         // VOP3 form of a VOP2 op
#define D8(D) "v_cvt_f32_u32 v" #D ", v1\n"              // VOP1
#define D9(D) "v_mov_b32_dpp v" #D ", v1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define D10(D) "v_cndmask_b32_e64 v" #D ", v1, v2, s[22:23]\n"
#define D11(D) "v_log_f32 v" #D ", v1\n"
#define D12(D) "v_add_u32 v" #D ", v1, v2\n"
#define D13(D) "v_fmac_f32 v" #D ", s20, v1\n"           // VOP2 fmac, SGPR
#define D14(D) "v_fma_f32 v" #D ", v1, v2, 1.0\n"        // VOP3, inline constant
#define D15(D) "v_mov_b32 v" #D ", s20\n"                // VOP1, SGPR
#define D16(D) "v_add_f32 v" #D ", v1, v2\n v_fma_f32 v" #D ", v1, s20, v2\n"   // mixed pair
#define D17(D) "v_rcp_f32 v" #D ", v1\n"
#define D18(D) "v_bitop3_b32 v" #D ", v1, v2, v9 bitop3:0x78\n"
#define MV(A, B) "v_mad_u64_u32 v[" #A ":" #B "], s[22:23], v1, v2, v[4:5]\n"    // all VGPR
#define MZ(A, B) "v_mad_u64_u32 v[" #A ":" #B "], s[22:23], v1, v2, 0\n"         // VGPR x VGPR + 0

#define F0(D) "v_or_b32 v" #D ", 0x3f800000, v1\n"       // VOP2 int, literal
#define F1(D) "v_and_b32 v" #D ", v1, v2\n"              // VOP2 int, VGPR
#define F2(D) "v_xor_b32 v" #D ", v1, v2\n"
#define F3(D) "v_lshlrev_b32 v" #D ", v1, v2\n"          // shift, VGPR amount
#define F4(D) "v_mul_lo_u32 v" #D ", v1, v2\n"
#define F5(D) "v_mul_hi_u32 v" #D ", v1, v2\n"
#define F6(D) "v_max_f32 v" #D ", v1, v2\n"
#define F7(D) "v_cvt_i32_f32 v" #D ", v1\n"
#define F8(D) "v_sub_u32 v" #D ", v1, v2\n"
#define F9(D) "v_bfe_u32 v" #D ", v1, v2, v3\n"
#define F10(D) "v_add3_u32 v" #D ", v1, v2, v3\n"
#define F11(D) "v_mul_u32_u24 v" #D ", v1, v2\n"
#define F12(D) "v_lshl_or_b32 v" #D ", v1, v2, v3\n"
#define F13(D) "v_perm_b32 v" #D ", v1, v2, v3\n"
#define F14(D) "v_rndne_f32 v" #D ", v1\n"
#define F15(D) "v_sqrt_f32 v" #D ", v1\n"
#define SH64(A, B) "v_lshlrev_b64 v[" #A ":" #B "], v1, v[2:3]\n"

#define G0(D) "v_cmp_gt_f32 vcc, v1, v2\n v_cndmask_b32 v" #D ", v1, v2, vcc\n"              // cmp -> cndmask (VCC)
#define G1(D) "v_cmp_gt_f32_e64 s[22:23], v1, v2\n v_cndmask_b32_e64 v" #D ", v1, v2, s[22:23]\n"   // via SGPR pair
#define G2(D) "v_cmp_gt_f32 vcc, v1, v2\n"                                             // cmp alone
#define G3(D) "v_max_f32 v" #D ", v1, v2\n v_min_f32 v" #D ", v" #D ", v3\n"          // max/min pair

#define KERNEL(NAME, BODY)                                                                            \
    __global__ __launch_bounds__(256) void NAME(unsigned long long *cyc) {                           \
        __syncthreads();                                                                              \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                  \
        asm volatile(INIT LOOP_HEAD BODY LOOP_TAIL "s_waitcnt lgkmcnt(0)\n" ::: CLOB);              \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                  \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;             \
    }

KERNEL(k0, R64(C0))
KERNEL(k1, R64(C1))
KERNEL(k2, R64(C2))
KERNEL(k3, R64(C3))
KERNEL(k4, R64(C4))
KERNEL(k5, R64(C5))
KERNEL(k6, R64(C6))
KERNEL(k7, R64(C7))
KERNEL(k8, R64(C8))
KERNEL(k9, R64(C9))
KERNEL(k10, R64(C10))
KERNEL(k11, R64(C11))
KERNEL(k12, R64(C12))
KERNEL(k13, R64(C13))
KERNEL(k14, R64(C14))
KERNEL(k15, R64(C15))
KERNEL(k16, P64(M64))
KERNEL(k17, P64(PKF))
KERNEL(k18, P64(PKA))

KERNEL(e0, R64(D0))
KERNEL(e1, R64(D1))
KERNEL(e2, R64(D2))
KERNEL(e3, R64(D3))
KERNEL(e4, R64(D4))
KERNEL(e5, R64(D5))
KERNEL(e6, R64(D6))
KERNEL(e7, R64(D7))
KERNEL(e8, R64(D8))
KERNEL(e9, R64(D9))
KERNEL(e10, R64(D10))
KERNEL(e11, R64(D11))
KERNEL(e12, R64(D12))
KERNEL(e13, R64(D13))
KERNEL(e14, R64(D14))
KERNEL(e15, R64(D15))
KERNEL(e16, R64(D16))
KERNEL(e17, R64(D17))
KERNEL(e18, R64(D18))
KERNEL(e19, P64(MV))
KERNEL(e20, P64(MZ))

KERNEL(f0, R64(F0))
KERNEL(f1, R64(F1))
KERNEL(f2, R64(F2))
KERNEL(f3, R64(F3))
KERNEL(f4, R64(F4))
KERNEL(f5, R64(F5))
KERNEL(f6, R64(F6))
KERNEL(f7, R64(F7))
KERNEL(f8, R64(F8))
KERNEL(f9, R64(F9))
KERNEL(f10, R64(F10))
KERNEL(f11, R64(F11))
KERNEL(f12, R64(F12))
KERNEL(f13, R64(F13))
KERNEL(f14, R64(F14))
KERNEL(f15, R64(F15))
KERNEL(f16, P64(SH64))

KERNEL(g0, R64(G0))
KERNEL(g1, R64(G1))
KERNEL(g2, R64(G2))
KERNEL(g3, R64(G3))

typedef void (*kfn)(unsigned long long *);
static const kfn K[] = {k0, k1, k2, k3, k4, k5, k6, k7, k8, k9, k10, k11, k12, k13, k14, k15, k16, k17, k18,
                        e0, e1, e2, e3, e4, e5, e6, e7, e8, e9, e10, e11, e12, e13, e14, e15, e16, e17, e18, e19, e20,
                        f0, f1, f2, f3, f4, f5, f6, f7, f8, f9, f10, f11, f12, f13, f14, f15, f16,
                        g0, g1, g2, g3};
static const char *N[] = {"fma v1,v2,v3 (banks 1,2,3)", "fma v4,v8,v12 (all bank 0)", "fma v4,v8,v1 (two bank 0)",
                          "fma v1,v1,v2 (src0==src1)", "fma v1,v2,v2 (src1==src2)", "fma v1,s20,v2 (SGPR)",
                          "add v1,v2", "add v4,v8 (same bank)", "bitop3 v1,v2,v3", "bitop3 v1,v2,s20",
                          "fmac v,v1,v2 (dst = src2)", "mul v1,v2", "fmamk v1,K,v2", "cndmask v1,v2,vcc",
                          "sin v1", "alignbit v1,v2,31", "mad_u64_u32 v1,s20", "pk_fma 3 pairs", "pk_add 2 pairs",
                          "add s20,v1 (VOP2 SGPR)", "add 1.0,v1 (VOP2 inline)", "mul lit,v1 (VOP2 literal)",
                          "lshlrev 6,v1 (VOP2 inline)", "xor s20,v1 (VOP2 SGPR)", "alignbit v1,v2,v3 (VGPR)",
                          "fma -v1,v2,v3 (modifier)", "mul_e64 v1,-v2", "cvt_f32_u32 v1", "mov_dpp quad_perm",
                          "cndmask_e64 v1,v2,s[22:23]", "log v1", "add_u32 v1,v2", "fmac s20,v1 (VOP2 SGPR)",
                          "fma v1,v2,1.0 (VOP3 inline)", "mov s20 (VOP1 SGPR)", "pair: add + fma(SGPR)",
                          "rcp v1", "bitop3 v1,v2,v9 (VGPR mask)", "mad_u64 v1,v2,v[4:5]", "mad_u64 v1,v2,0",
                          "or lit,v1", "and v1,v2", "xor v1,v2", "lshlrev v1,v2", "mul_lo_u32", "mul_hi_u32",
                          "max_f32", "cvt_i32_f32", "sub_u32", "bfe_u32", "add3_u32", "mul_u32_u24",
                          "lshl_or_b32", "perm_b32", "rndne_f32", "sqrt_f32", "lshlrev_b64",
                          "pair: cmp vcc + cndmask vcc", "pair: cmp_e64 s + cndmask_e64 s", "cmp vcc alone",
                          "pair: max + min"};

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned long long *d;
    (void)hipMalloc(&d, (size_t)cus * 4 * 4 * 8);
    std::vector<unsigned long long> c;
    printf("SIMD cycles per wave64 instruction, median over waves (w = waves per SIMD)\n");
    for (int k = 0; k < (int)(sizeof(K) / sizeof(K[0])); ++k) {
        printf("%-30s", N[k]);
        for (int w = 1; w <= 4; w *= 2) {
            const int blocks = cus * w;   // 4 waves per block, one per SIMD: w waves per SIMD
            hipLaunchKernelGGL(K[k], dim3(blocks), dim3(256), 0, 0, d);
            hipLaunchKernelGGL(K[k], dim3(blocks), dim3(256), 0, 0, d);
            (void)hipDeviceSynchronize();
            c.resize((size_t)blocks * 4);
            (void)hipMemcpy(c.data(), d, c.size() * 8, hipMemcpyDeviceToHost);
            std::sort(c.begin(), c.end());
            const double med = (double)c[c.size() / 2];
            printf("  w%d %6.2f", w, med / (64.0 * ITERS) / w);
        }
        printf("\n");
    }
    return 0;
}
