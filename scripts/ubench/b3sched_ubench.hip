// Microbenchmark: BLAKE3 compressions per second for each half-round schedule of
// scripts/b3_sched_gen.py (order of the four G's instructions x s_nop policy), every half-round one
// asm block so the generated order is the issued order. 680 VALU per compression.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define KB_PROLOGUE                                                                                  \
    uint32_t s0 = threadIdx.x, s1 = s0 * 3, s2 = s0 * 5, s3 = s0 * 7, s4 = s0 + 1, s5 = s0 + 2,      \
             s6 = s0 + 3, s7 = s0 + 4, s8 = s0 ^ 9, s9 = s0 ^ 10, s10 = s0 ^ 11, s11 = s0 ^ 12,      \
             s12 = s0 * 13, s13 = s0 * 17, s14 = s0 * 19, s15 = s0 * 23;                             \
    uint32_t m[16];                                                                                  \
    _Pragma("unroll") for (int i = 0; i < 16; i++) m[i] = blockIdx.x * 16 + i;
#define B3_COL_OPS                                                                                   \
    "+v"(s0), "+v"(s4), "+v"(s8), "+v"(s12), "+v"(s1), "+v"(s5), "+v"(s9), "+v"(s13), "+v"(s2),       \
        "+v"(s6), "+v"(s10), "+v"(s14), "+v"(s3), "+v"(s7), "+v"(s11), "+v"(s15)                     \
    : "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]), "v"(m[6]), "v"(m[7])
#define B3_DIAG_OPS                                                                                  \
    "+v"(s0), "+v"(s5), "+v"(s10), "+v"(s15), "+v"(s1), "+v"(s6), "+v"(s11), "+v"(s12), "+v"(s2),     \
        "+v"(s7), "+v"(s8), "+v"(s13), "+v"(s3), "+v"(s4), "+v"(s9), "+v"(s14)                       \
    : "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(m[11]), "v"(m[12]), "v"(m[13]), "v"(m[14]), "v"(m[15])
#define B3_PERMUTE_M                                                                                 \
    do {                                                                                             \
        uint32_t t[16];                                                                              \
        _Pragma("unroll") for (int i = 0; i < 16; i++) t[i] = m[i];                                  \
        const int P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};                    \
        _Pragma("unroll") for (int i = 0; i < 16; i++) m[i] = t[P[i]];                               \
    } while (0)
#define KB_OUT_XOR                                                                                   \
    s0 ^= s8; s1 ^= s9; s2 ^= s10; s3 ^= s11; s4 ^= s12; s5 ^= s13; s6 ^= s14; s7 ^= s15;
#define KB_EPILOGUE                                                                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                                                     \
        s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7 ^ s8 ^ s9 ^ s10 ^ s11 ^ s12 ^ s13 ^ s14 ^ s15;
#include "b3sched_gen.inc"

int main(int argc, char** argv) {
    uint32_t* d;
    const int threads = 256, iters = argc > 1 ? atoi(argv[1]) : 64;  // 64: ~1 ms per launch at 8 waves
    (void)hipMalloc(&d, (size_t)256 * 8 * threads * 4);
    const int waves_per_simd[] = {4, 5, 6, 8};
    for (auto& k : kbs) hipLaunchKernelGGL(k.f, dim3(2048), dim3(threads), 0, 0, d, iters);  // clocks up
    (void)hipDeviceSynchronize();
    printf("%-16s", "schedule \\ waves");
    for (int w : waves_per_simd) printf("  %6d", w);
    printf("   (T lane-instr/s at 680 per compression)\n");
    for (auto& k : kbs) {
        printf("%-16s", k.n);
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
            printf("  %6.1f", (double)blocks * threads * iters * 680 / ms / 1e9);
        }
        printf("\n");
    }
    return 0;
}
