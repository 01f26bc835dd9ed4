// Microbenchmark: wave64 issue throughput of the integer VALU instructions used by BLAKE3 and the
// Goldilocks field code on gfx950 (8 independent chains per lane, 8 waves per SIMD)
#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP8(X) X X X X X X X X
#define DEF(NAME, ASM)                                                                           \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {                    \
        unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 2, \
                 a6 = a0 + 3, a7 = a0 + 4, k = blockIdx.x | 1;                                  \
        for (int it = 0; it < iters; it++) {                                                     \
            REP8(asm volatile(ASM : "+v"(a0) : "v"(k) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a1) : "v"(k) : "vcc", "s40", "s41");   \
                 asm volatile(ASM : "+v"(a2) : "v"(k) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a3) : "v"(k) : "vcc", "s40", "s41");   \
                 asm volatile(ASM : "+v"(a4) : "v"(k) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a5) : "v"(k) : "vcc", "s40", "s41");   \
                 asm volatile(ASM : "+v"(a6) : "v"(k) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a7) : "v"(k) : "vcc", "s40", "s41");)  \
        }                                                                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
    }
DEF(k_add, "v_add_u32 %0, %0, %1")
DEF(k_xor, "v_xor_b32 %0, %0, %1")
DEF(k_add3, "v_add3_u32 %0, %0, %1, %0")
DEF(k_alignbit, "v_alignbit_b32 %0, %0, %0, 16")
DEF(k_xad, "v_xad_u32 %0, %0, %1, %0")
DEF(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
DEF(k_perm, "v_perm_b32 %0, %0, %1, %1")
DEF(k_mad32, "v_mad_u32_u24 %0, %0, %1, %0")
DEF(k_mullo, "v_mul_lo_u32 %0, %0, %1")
DEF(k_mulhi, "v_mul_hi_u32 %0, %0, %1")
DEF(k_addco, "v_add_co_u32 %0, vcc, %0, %1")
DEF(k_lshl_or, "v_lshl_or_b32 %0, %0, 7, %1")
DEF(k_sdwa_xor, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
DEF(k_sdwa_add, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
DEF(k_cndmask, "v_cndmask_b32_e32 %0, %0, %1, vcc")
DEF(k_lshrrev, "v_lshrrev_b32_e32 %0, 7, %0")
// 64-bit register-pair forms (Goldilocks add / compare / multiply lowering)
#define DEF64(NAME, ASM)                                                                         \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {                    \
        unsigned long long a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1,  \
                           a5 = a0 + 2, a6 = a0 + 3, a7 = a0 + 4, k = blockIdx.x | 1;           \
        unsigned k32 = blockIdx.x | 1;                                                            \
        for (int it = 0; it < iters; it++) {                                                     \
            REP8(asm volatile(ASM : "+v"(a0) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a1) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); \
                 asm volatile(ASM : "+v"(a2) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a3) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); \
                 asm volatile(ASM : "+v"(a4) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a5) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); \
                 asm volatile(ASM : "+v"(a6) : "v"(k), "v"(k32) : "vcc", "s40", "s41"); asm volatile(ASM : "+v"(a7) : "v"(k), "v"(k32) : "vcc", "s40", "s41");) \
        }                                                                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    }
DEF64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %1")
DEF64(k_cmp64, "v_cmp_lt_u64_e32 vcc, %0, %1")
DEF64(k_mad64, "v_mad_u64_u32 %0, vcc, %2, %2, %0")
DEF64(k_lshl64, "v_lshlrev_b64 %0, 7, %0")
DEF64(k_mov64, "v_mov_b64 %0, %1")
DEF(k_subco, "v_sub_co_u32_e64 %0, vcc, %0, %1")
DEF(k_subb, "v_subb_co_u32_e32 %0, vcc, %0, %1, vcc")
DEF(k_cnd64, "v_cndmask_b32_e64 %0, %0, %1, vcc")
DEF(k_mov, "v_mov_b32 %0, %1")
DEF(k_addc, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
DEF(k_cmp32, "v_cmp_lt_u32_e32 vcc, %0, %1")
DEF(k_sub, "v_sub_u32 %0, %0, %1")
DEF(k_and, "v_and_b32 %0, %0, %1")
DEF(k_mul24, "v_mul_u32_u24 %0, %0, %1")
DEF(k_addco_s, "v_add_co_u32_e64 %0, s[40:41], %0, %1")
DEF(k_addc_s, "v_addc_co_u32_e64 %0, s[40:41], %0, %1, s[40:41]")
DEF(k_lshl_add32, "v_lshl_add_u32 %0, %0, 3, %1")
DEF(k_cnd_s, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
DEF(k_bfe, "v_bfe_u32 %0, %0, 8, 16")
DEF64(k_lshr64, "v_lshrrev_b64 %0, 7, %0")
DEF64(k_mulhi64a, "v_mad_u64_u32 %0, s[40:41], %2, %2, %0")
// round 5: bitop3 forms (three distinct sources, two-input xor) and three-input xor / or
DEF(k_bitop3_3, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")
DEF(k_bitop3_x2, "v_bitop3_b32 %0, %0, %1, 0 bitop3:0x66")
DEF(k_or3, "v_or3_b32 %0, %0, %1, %0")
DEF(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
DEF(k_alignbit2, "v_alignbit_b32 %0, %0, %1, 16")
DEF(k_pk_add16, "v_pk_add_u16 %0, %0, %1")
// VOP2 (e32) against VOP3 (e64) encodings of the same operation
DEF(k_add_e64, "v_add_u32_e64 %0, %0, %1")
DEF(k_sub_e64, "v_sub_u32_e64 %0, %0, %1")
DEF(k_and_e64, "v_and_b32_e64 %0, %0, %1")
DEF(k_lshr_e64, "v_lshrrev_b32_e64 %0, 7, %0")
DEF(k_mov_e64, "v_mov_b32_e64 %0, %1")
DEF(k_subco_e32, "v_sub_co_u32_e32 %0, vcc, %0, %1")
DEF(k_subco_e64s, "v_sub_co_u32_e64 %0, s[40:41], %0, %1")
DEF(k_cnd_vcc64, "v_cndmask_b32_e64 %0, %0, %1, vcc")

int main() {
    unsigned* d;
    const int blocks = 256 * 8, threads = 256, iters = 2048;
    hipMalloc(&d, (size_t)blocks * threads * 4);
    struct { const char* n; void (*f)(unsigned*, int); } ks[] = {
        {"v_add_u32", k_add}, {"v_xor_b32", k_xor}, {"v_add3_u32", k_add3}, {"v_alignbit_b32", k_alignbit},
        {"v_xad_u32", k_xad}, {"v_bitop3_b32", k_bitop3}, {"v_perm_b32", k_perm}, {"v_mad_u32_u24", k_mad32},
        {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi}, {"v_add_co_u32", k_addco}, {"v_lshl_or_b32", k_lshl_or},
        {"v_xor_b32_sdwa", k_sdwa_xor}, {"v_add_u32_sdwa", k_sdwa_add}, {"v_cndmask_b32", k_cndmask},
        {"v_lshrrev_b32", k_lshrrev}, {"v_lshl_add_u64", k_lshladd64}, {"v_cmp_lt_u64", k_cmp64},
        {"v_mad_u64_u32", k_mad64}, {"v_lshlrev_b64", k_lshl64}, {"v_mov_b64", k_mov64}, {"v_sub_co_u32_e64", k_subco},
        {"v_subb_co_u32", k_subb}, {"v_cndmask_b32_e64", k_cnd64}, {"v_mov_b32", k_mov},
        {"v_addc_co_u32", k_addc}, {"v_cmp_lt_u32", k_cmp32}, {"v_sub_u32", k_sub}, {"v_and_b32", k_and},
        {"v_mul_u32_u24", k_mul24}, {"v_add_co_u32_e64 s", k_addco_s}, {"v_addc_co_u32_e64 s", k_addc_s},
        {"v_lshl_add_u32", k_lshl_add32}, {"v_cndmask_e64 s", k_cnd_s}, {"v_bfe_u32", k_bfe},
        {"v_lshrrev_b64", k_lshr64}, {"v_mad_u64_u32 s", k_mulhi64a}, {"v_bitop3 3src", k_bitop3_3},
        {"v_bitop3 xor2", k_bitop3_x2}, {"v_or3_b32", k_or3}, {"v_xor_b32_e64", k_xor_e64},
        {"v_alignbit 2src", k_alignbit2}, {"v_pk_add_u16", k_pk_add16}, {"v_add_u32_e64", k_add_e64},
        {"v_sub_u32_e64", k_sub_e64}, {"v_and_b32_e64", k_and_e64}, {"v_lshrrev_b32_e64", k_lshr_e64},
        {"v_mov_b32_e64", k_mov_e64}, {"v_sub_co_u32_e32", k_subco_e32}, {"v_sub_co_u32_e64 s", k_subco_e64s},
        {"v_cndmask_e64 vcc", k_cnd_vcc64}};
    for (auto& k : ks) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float ms = 0;
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        double ops = (double)blocks * threads * iters * 64;
        printf("%-16s %.3f ms  %.1f T lane-ops/s\n", k.n, ms, ops / ms / 1e9);
    }
    return 0;
}
