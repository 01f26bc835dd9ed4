// Microbenchmark: how gfx950 issues a MIX of fast (two-source e64 xor) and slow (alignbit) VALU
// instructions -- grouped, interleaved, dependent -- and how the fast rate depends on the number of
// independent chains and of waves per SIMD. Rates in T lane-ops/s over all instructions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define F(x) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(k))
#define S(x) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x))
#define A(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(k))
#define A3(x) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(k))
#define X32(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k))
#define KERN(NAME, OPS, BODY)                                                                     \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {                     \
        unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 2, \
                 a6 = a0 + 3, a7 = a0 + 4, k = blockIdx.x | 1;                                   \
        for (int it = 0; it < iters; it++) { BODY BODY BODY BODY }                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;        \
    }                                                                                            \
    static const int NAME##_ops = 4 * (OPS);
KERN(k_f8, 16, F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7); F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);)
KERN(k_s8, 16, S(a0); S(a1); S(a2); S(a3); S(a4); S(a5); S(a6); S(a7); S(a0); S(a1); S(a2); S(a3); S(a4); S(a5); S(a6); S(a7);)
KERN(k_f8s8, 16, F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7); S(a0); S(a1); S(a2); S(a3); S(a4); S(a5); S(a6); S(a7);)
KERN(k_f4s4, 16, F(a0); F(a1); F(a2); F(a3); S(a4); S(a5); S(a6); S(a7); F(a4); F(a5); F(a6); F(a7); S(a0); S(a1); S(a2); S(a3);)
KERN(k_f2s2, 16, F(a0); F(a1); S(a2); S(a3); F(a4); F(a5); S(a6); S(a7); S(a0); S(a1); F(a2); F(a3); S(a4); S(a5); F(a6); F(a7);)
KERN(k_f1s1, 16, F(a0); S(a1); F(a2); S(a3); F(a4); S(a5); F(a6); S(a7); S(a0); F(a1); S(a2); F(a3); S(a4); F(a5); S(a6); F(a7);)
KERN(k_dep, 16, F(a0); S(a0); F(a1); S(a1); F(a2); S(a2); F(a3); S(a3); F(a4); S(a4); F(a5); S(a5); F(a6); S(a6); F(a7); S(a7);)
KERN(k_fc1, 8, F(a0); F(a0); F(a0); F(a0); F(a0); F(a0); F(a0); F(a0);)
KERN(k_fc2, 8, F(a0); F(a1); F(a0); F(a1); F(a0); F(a1); F(a0); F(a1);)
KERN(k_fc4, 8, F(a0); F(a1); F(a2); F(a3); F(a0); F(a1); F(a2); F(a3);)
KERN(k_sc1, 8, S(a0); S(a0); S(a0); S(a0); S(a0); S(a0); S(a0); S(a0);)
KERN(k_sc2, 8, S(a0); S(a1); S(a0); S(a1); S(a0); S(a1); S(a0); S(a1);)
KERN(k_x32c1, 8, X32(a0); X32(a0); X32(a0); X32(a0); X32(a0); X32(a0); X32(a0); X32(a0);)
KERN(k_x32c8, 8, X32(a0); X32(a1); X32(a2); X32(a3); X32(a4); X32(a5); X32(a6); X32(a7);)
// the G column step's op mix: per G 2 add3, 2 add, 4 xor, 4 rotate; four independent G's as 8 chains
KERN(k_gmix, 24, A3(a0); A3(a1); A3(a2); A3(a3); F(a4); F(a5); F(a6); F(a7); S(a4); S(a5); S(a6); S(a7);
     A(a0); A(a1); A(a2); A(a3); F(a4); F(a5); F(a6); F(a7); S(a4); S(a5); S(a6); S(a7);)
KERN(k_gmix_pairs, 24, A3(a0); A3(a1); F(a4); F(a5); A3(a2); A3(a3); F(a6); F(a7); S(a4); S(a5); S(a6); S(a7);
     A(a0); A(a1); A(a2); A(a3); F(a4); F(a5); F(a6); F(a7); S(a4); S(a5); S(a6); S(a7);)

int main() {
    unsigned* d;
    const int threads = 256, iters = 512;
    hipMalloc(&d, (size_t)2048 * threads * 4);
    struct { const char* n; void (*f)(unsigned*, int); int ops; } ks[] = {
        {"f8 (8 chains)", k_f8, k_f8_ops}, {"s8 (8 chains)", k_s8, k_s8_ops}, {"f8 then s8", k_f8s8, k_f8s8_ops},
        {"f4 s4", k_f4s4, k_f4s4_ops}, {"f2 s2", k_f2s2, k_f2s2_ops}, {"f1 s1", k_f1s1, k_f1s1_ops},
        {"f->s dependent", k_dep, k_dep_ops}, {"f 1 chain", k_fc1, k_fc1_ops}, {"f 2 chains", k_fc2, k_fc2_ops},
        {"f 4 chains", k_fc4, k_fc4_ops}, {"s 1 chain", k_sc1, k_sc1_ops}, {"s 2 chains", k_sc2, k_sc2_ops},
        {"xor e32 1 chain", k_x32c1, k_x32c1_ops}, {"xor e32 8 chains", k_x32c8, k_x32c8_ops},
        {"G mix", k_gmix, k_gmix_ops}, {"G mix paired", k_gmix_pairs, k_gmix_pairs_ops}};
    const int waves_per_simd[] = {1, 2, 4, 8};
    printf("%-18s", "pattern \\ waves/SIMD");
    for (int w : waves_per_simd) printf("  %6d", w);
    printf("   (T lane-ops/s)\n");
    for (auto& k : ks) {
        printf("%-18s", k.n);
        for (int w : waves_per_simd) {
            int blocks = 256 * w;
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
            double ops = (double)blocks * threads * iters * k.ops;
            printf("  %6.1f", ops / ms / 1e9);
        }
        printf("\n");
    }
    return 0;
}
