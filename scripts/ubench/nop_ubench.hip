// Microbenchmark: does an s_nop between VALU instructions of one wave change the issue rate of a
// fast/slow mix on gfx950? Each pattern is ONE asm block (the compiler inserts nothing inside it),
// 16 VALU over 8 independent registers, optionally with `s_nop 0` after chosen instructions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define F(i) "v_xor_b32_e64 %" #i ", %" #i ", %8\n"
#define S(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 16\n"
#define N "s_nop 0\n"
#define KERN(NAME, BODY)                                                                            \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {                      \
        unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 2,  \
                 a6 = a0 + 3, a7 = a0 + 4, k = blockIdx.x | 1;                                    \
        for (int it = 0; it < iters; it++)                                                        \
            asm volatile(BODY BODY BODY BODY                                                      \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(k));                                                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;         \
    }
KERN(k_f16, F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7))
KERN(k_s16, S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7))
KERN(k_f1s1, F(0) S(1) F(2) S(3) F(4) S(5) F(6) S(7) S(0) F(1) S(2) F(3) S(4) F(5) S(6) F(7))
KERN(k_f1s1_nall, F(0) N S(1) N F(2) N S(3) N F(4) N S(5) N F(6) N S(7) N S(0) N F(1) N S(2) N F(3) N S(4) N F(5) N S(6) N F(7) N)
KERN(k_f1s1_nafs, F(0) N S(1) F(2) N S(3) F(4) N S(5) F(6) N S(7) S(0) F(1) N S(2) F(3) N S(4) F(5) N S(6) F(7) N)
KERN(k_f1s1_nasf, F(0) S(1) N F(2) S(3) N F(4) S(5) N F(6) S(7) N S(0) N F(1) S(2) N F(3) S(4) N F(5) S(6) N F(7))
KERN(k_dep, F(0) S(0) F(1) S(1) F(2) S(2) F(3) S(3) F(4) S(4) F(5) S(5) F(6) S(6) F(7) S(7))
KERN(k_dep_n, F(0) N S(0) F(1) N S(1) F(2) N S(2) F(3) N S(3) F(4) N S(4) F(5) N S(5) F(6) N S(6) F(7) N S(7))
KERN(k_f8s8, F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7))
KERN(k_f2s2, F(0) F(1) S(2) S(3) F(4) F(5) S(6) S(7) S(0) S(1) F(2) F(3) S(4) S(5) F(6) F(7))
KERN(k_f16_n, F(0) N F(1) N F(2) N F(3) N F(4) N F(5) N F(6) N F(7) N F(0) N F(1) N F(2) N F(3) N F(4) N F(5) N F(6) N F(7) N)
KERN(k_s16_n, S(0) N S(1) N S(2) N S(3) N S(4) N S(5) N S(6) N S(7) N S(0) N S(1) N S(2) N S(3) N S(4) N S(5) N S(6) N S(7) N)

int main() {
    unsigned* d;
    const int threads = 256, iters = 512;
    (void)hipMalloc(&d, (size_t)256 * 8 * threads * 4);
    struct { const char* n; void (*f)(unsigned*, int); } ks[] = {
        {"f16", k_f16}, {"s16", k_s16}, {"f1s1", k_f1s1}, {"f1s1 nop all", k_f1s1_nall},
        {"f1s1 nop after f", k_f1s1_nafs}, {"f1s1 nop after s", k_f1s1_nasf}, {"f->s dep", k_dep},
        {"f->s dep nop", k_dep_n}, {"f8s8", k_f8s8}, {"f2s2", k_f2s2}, {"f16 nop all", k_f16_n},
        {"s16 nop all", k_s16_n}};
    const int waves_per_simd[] = {1, 2, 4, 5, 8};
    printf("%-18s", "pattern \\ waves");
    for (int w : waves_per_simd) printf("  %6d", w);
    printf("   (T lane-VALU/s, nops not counted)\n");
    for (auto& k : ks) {
        printf("%-18s", k.n);
        for (int w : waves_per_simd) {
            int blocks = 256 * w;
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            float ms = 0;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, iters);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms, a, b);
            }
            double ops = (double)blocks * threads * iters * 64;
            printf("  %6.1f", ops / ms / 1e9);
        }
        printf("\n");
    }
    return 0;
}
