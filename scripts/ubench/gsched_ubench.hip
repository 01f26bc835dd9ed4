// Microbenchmark: instruction ORDER of the BLAKE3 round on gfx950. Seven rounds (column + diagonal
// G's) over a 16-word state with 16 message words in registers, every instruction a volatile asm
// statement so the written order is the issued order; the variants differ only in how the four
// independent G functions of a half-round are interleaved. 680 VALU per compression as in the
// product (224 xor, 224 rotate, 112 add3, 112 add, 8 output xors).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ADD3(a, b, m) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(m))
#define ADD(c, d) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(c) : "v"(d))
#define XOR(d, a) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(d) : "v"(a))
#define ROT(d, n) asm volatile("v_alignbit_b32 %0, %0, %0, " #n : "+v"(d))

// the twelve steps of G as six (op, op) pieces: 0 add3, 1 xor, 2 rot16, 3 add, 4 xor, 5 rot12,
// 6 add3, 7 xor, 8 rot8, 9 add, 10 xor, 11 rot7
#define STEP(k, a, b, c, d, x, y)                  \
    do {                                           \
        switch (k) {                               \
            case 0: ADD3(a, b, x); break;          \
            case 1: XOR(d, a); break;              \
            case 2: ROT(d, 16); break;             \
            case 3: ADD(c, d); break;              \
            case 4: XOR(b, c); break;              \
            case 5: ROT(b, 12); break;             \
            case 6: ADD3(a, b, y); break;          \
            case 7: XOR(d, a); break;              \
            case 8: ROT(d, 8); break;              \
            case 9: ADD(c, d); break;              \
            case 10: XOR(b, c); break;             \
            case 11: ROT(b, 7); break;             \
        }                                          \
    } while (0)

// ORDER 0: G by G (each G's twelve steps back to back)
// ORDER 1: lockstep (step k of all four G's, then step k+1)
// ORDER 2: two pairs (G0/G1 interleaved step by step, then G2/G3)
// ORDER 3: lockstep, but every xor immediately followed by its rotate (xor g, rot g for g = 0..3)
// ORDER 4: lockstep by pairs of steps within two G's: (G0 k, G1 k, G0 k+1, G1 k+1 ...) for G0/G1 and
//          G2/G3 alternating every two steps
#define HALF(ORDER, A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3, m0, m1, m2, m3, m4, m5, m6, m7) \
    do {                                                                                   \
        if (ORDER == 0) {                                                                  \
            _Pragma("unroll") for (int k = 0; k < 12; k++) STEP(k, A0, B0, C0, D0, m0, m1); \
            _Pragma("unroll") for (int k = 0; k < 12; k++) STEP(k, A1, B1, C1, D1, m2, m3); \
            _Pragma("unroll") for (int k = 0; k < 12; k++) STEP(k, A2, B2, C2, D2, m4, m5); \
            _Pragma("unroll") for (int k = 0; k < 12; k++) STEP(k, A3, B3, C3, D3, m6, m7); \
        } else if (ORDER == 1) {                                                           \
            _Pragma("unroll") for (int k = 0; k < 12; k++) {                               \
                STEP(k, A0, B0, C0, D0, m0, m1); STEP(k, A1, B1, C1, D1, m2, m3);          \
                STEP(k, A2, B2, C2, D2, m4, m5); STEP(k, A3, B3, C3, D3, m6, m7);          \
            }                                                                              \
        } else if (ORDER == 2) {                                                           \
            _Pragma("unroll") for (int k = 0; k < 12; k++) {                               \
                STEP(k, A0, B0, C0, D0, m0, m1); STEP(k, A1, B1, C1, D1, m2, m3);          \
            }                                                                              \
            _Pragma("unroll") for (int k = 0; k < 12; k++) {                               \
                STEP(k, A2, B2, C2, D2, m4, m5); STEP(k, A3, B3, C3, D3, m6, m7);          \
            }                                                                              \
        } else if (ORDER == 3) {                                                           \
            _Pragma("unroll") for (int k = 0; k < 12; k += 3) {                            \
                STEP(k, A0, B0, C0, D0, m0, m1); STEP(k, A1, B1, C1, D1, m2, m3);          \
                STEP(k, A2, B2, C2, D2, m4, m5); STEP(k, A3, B3, C3, D3, m6, m7);          \
                STEP(k + 1, A0, B0, C0, D0, m0, m1); STEP(k + 2, A0, B0, C0, D0, m0, m1);  \
                STEP(k + 1, A1, B1, C1, D1, m2, m3); STEP(k + 2, A1, B1, C1, D1, m2, m3);  \
                STEP(k + 1, A2, B2, C2, D2, m4, m5); STEP(k + 2, A2, B2, C2, D2, m4, m5);  \
                STEP(k + 1, A3, B3, C3, D3, m6, m7); STEP(k + 2, A3, B3, C3, D3, m6, m7);  \
            }                                                                              \
        } else {                                                                           \
            _Pragma("unroll") for (int k = 0; k < 12; k += 2) {                            \
                STEP(k, A0, B0, C0, D0, m0, m1); STEP(k, A1, B1, C1, D1, m2, m3);          \
                STEP(k + 1, A0, B0, C0, D0, m0, m1); STEP(k + 1, A1, B1, C1, D1, m2, m3);  \
                STEP(k, A2, B2, C2, D2, m4, m5); STEP(k, A3, B3, C3, D3, m6, m7);          \
                STEP(k + 1, A2, B2, C2, D2, m4, m5); STEP(k + 1, A3, B3, C3, D3, m6, m7);  \
            }                                                                              \
        }                                                                                  \
    } while (0)

template <int ORDER>
__global__ __launch_bounds__(256) void kg(uint32_t* out, int iters) {
    uint32_t s0 = threadIdx.x, s1 = s0 * 3, s2 = s0 * 5, s3 = s0 * 7, s4 = s0 + 1, s5 = s0 + 2, s6 = s0 + 3,
             s7 = s0 + 4, s8 = s0 ^ 9, s9 = s0 ^ 10, s10 = s0 ^ 11, s11 = s0 ^ 12, s12 = s0 * 13, s13 = s0 * 17,
             s14 = s0 * 19, s15 = s0 * 23;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = blockIdx.x * 16 + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 7; r++) {
            HALF(ORDER, s0, s4, s8, s12, s1, s5, s9, s13, s2, s6, s10, s14, s3, s7, s11, s15, m[0], m[1], m[2],
                 m[3], m[4], m[5], m[6], m[7]);
            HALF(ORDER, s0, s5, s10, s15, s1, s6, s11, s12, s2, s7, s8, s13, s3, s4, s9, s14, m[8], m[9], m[10],
                 m[11], m[12], m[13], m[14], m[15]);
        }
        XOR(s0, s8); XOR(s1, s9); XOR(s2, s10); XOR(s3, s11); XOR(s4, s12); XOR(s5, s13); XOR(s6, s14);
        XOR(s7, s15);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7 ^ s8 ^ s9 ^ s10 ^ s11 ^ s12 ^ s13 ^ s14 ^ s15;
}

int main() {
    uint32_t* d;
    const int threads = 256, iters = 64;
    (void)hipMalloc(&d, (size_t)256 * 8 * threads * 4);
    struct { const char* n; void (*f)(uint32_t*, int); } ks[] = {
        {"G by G", kg<0>}, {"lockstep", kg<1>}, {"two pairs", kg<2>}, {"lockstep xor+rot", kg<3>},
        {"pairs of steps", kg<4>}};
    const int waves_per_simd[] = {2, 4, 5, 6, 8};
    printf("%-18s", "order \\ waves/SIMD");
    for (int w : waves_per_simd) printf("  %6d", w);
    printf("   (T lane-instr/s at 680 per compression)\n");
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
            double ops = (double)blocks * threads * iters * 680;
            printf("  %6.1f", ops / ms / 1e9);
        }
        printf("\n");
    }
    return 0;
}
