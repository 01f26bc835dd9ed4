// Microbenchmark: Goldilocks multiply/add throughput on gfx950 (independent chains per thread).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../xfg-stark_amd/csrc/gl.hpp"
using namespace xfg;

__device__ __forceinline__ u64 mul_v2(u64 a, u64 b) {
    u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    u64 p00 = (u64)a0 * b0;
    u64 t1 = (u64)a0 * b1 + (p00 >> 32);
    u64 t2 = (u64)a1 * b0 + (u32)t1;
    u64 lo = (u64)(u32)p00 | ((u64)(u32)t2 << 32);
    u64 hi = (u64)a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    return gl_reduce(hi, lo);
}
// inline-asm reduction using carry flags directly
__device__ __forceinline__ u64 reduce_asm(u64 hi, u64 lo) {
    u32 lx = (u32)lo, ly = (u32)(lo >> 32), hl = (u32)hi, hh = (u32)(hi >> 32);
    u32 t0x, t0y, ttx, tty, m, rx, ry, cx, cy;
    asm volatile(
        "v_sub_co_u32 %0, vcc, %9, %12\n\t"
        "v_subbrev_co_u32 %1, vcc, 0, %10, vcc\n\t"
        "v_cndmask_b32 %4, 0, -1, vcc\n\t"
        "v_sub_co_u32 %0, vcc, %0, %4\n\t"
        "v_subbrev_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_sub_co_u32 %2, vcc, 0, %11\n\t"
        "v_subbrev_co_u32 %3, vcc, 0, %11, vcc\n\t"
        "v_add_co_u32 %5, vcc, %0, %2\n\t"
        "v_addc_co_u32 %6, vcc, %1, %3, vcc\n\t"
        "v_cndmask_b32 %4, 0, -1, vcc\n\t"
        "v_add_co_u32 %5, vcc, %5, %4\n\t"
        "v_addc_co_u32 %6, vcc, %6, 0, vcc\n\t"
        "v_add_co_u32 %7, vcc, %5, -1\n\t"
        "v_addc_co_u32 %8, vcc, %6, 0, vcc\n\t"
        "v_cndmask_b32 %5, %5, %7, vcc\n\t"
        "v_cndmask_b32 %6, %6, %8, vcc\n\t"
        : "=&v"(t0x), "=&v"(t0y), "=&v"(ttx), "=&v"(tty), "=&v"(m), "=&v"(rx), "=&v"(ry), "=&v"(cx), "=&v"(cy)
        : "v"(lx), "v"(ly), "v"(hl), "v"(hh)
        : "vcc");
    return ((u64)ry << 32) | rx;
}
__device__ __forceinline__ u64 mul_v3(u64 a, u64 b) {
    u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    u64 p00 = (u64)a0 * b0;
    u64 t1 = (u64)a0 * b1 + (p00 >> 32);
    u64 t2 = (u64)a1 * b0 + (u32)t1;
    u64 lo = (u64)(u32)p00 | ((u64)(u32)t2 << 32);
    u64 hi = (u64)a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    return reduce_asm(hi, lo);
}

__device__ __forceinline__ u64 add_v2(u64 a, u64 b) {
    u64 q = P - b;            // in [1, P]
    u64 d = a - q;
    return (a < q) ? d - EPS : d;   // borrow: d + P == d - EPS (mod 2^64)
}
template <int V>
__global__ __launch_bounds__(256) void kmul(u64* out, u64 seed, int iters) {
    u64 x[8], w = seed | 1;
    for (int k = 0; k < 8; k++) x[k] = (seed * (threadIdx.x + 1 + 77 * k)) % P;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (V == 0) x[k] = gl_mul(x[k], w);
            else if (V == 1) x[k] = mul_v2(x[k], w);
            else if (V == 2) x[k] = mul_v3(x[k], w);
            else if (V == 3) x[k] = gl_add(x[k], w);
            else if (V == 5) x[k] = add_v2(x[k], w);
            else x[k] = gl_sub(x[k], w);
        }
    }
    u64 s = 0;
    for (int k = 0; k < 8; k++) s ^= x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    u64* d;
    const int blocks = 256 * 16, threads = 256, iters = 512;
    hipMalloc(&d, (size_t)blocks * threads * 8);
    const char* names[] = {"gl_mul (current)", "mul_v2 (4 mad)", "mul_v3 (4 mad + asm reduce)", "gl_add", "gl_sub", "add_v2 (a-(P-b))"};
    for (int v = 0; v < 6; v++) {
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            switch (v) {
                case 0: hipLaunchKernelGGL(kmul<0>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
                case 1: hipLaunchKernelGGL(kmul<1>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
                case 2: hipLaunchKernelGGL(kmul<2>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
                case 3: hipLaunchKernelGGL(kmul<3>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
                case 4: hipLaunchKernelGGL(kmul<4>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
                case 5: hipLaunchKernelGGL(kmul<5>, dim3(blocks), dim3(threads), 0, 0, d, 12345, iters); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        double ops = (double)blocks * threads * iters * 8;
        printf("%-30s %8.3f ms  %7.1f G ops/s  (%.2f ns/op/CU-equiv)\n", names[v], ms, ops / ms / 1e6,
               ms * 1e6 / (ops / 256));
    }
    // correctness of variants
    u64 h0[1], h1[1], h2[1];
    hipLaunchKernelGGL(kmul<0>, dim3(1), dim3(1), 0, 0, d, 999, 100); hipMemcpy(h0, d, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(kmul<1>, dim3(1), dim3(1), 0, 0, d, 999, 100); hipMemcpy(h1, d, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(kmul<2>, dim3(1), dim3(1), 0, 0, d, 999, 100); hipMemcpy(h2, d, 8, hipMemcpyDeviceToHost);
    u64 h3[1], h4[1];
    hipLaunchKernelGGL(kmul<3>, dim3(1), dim3(1), 0, 0, d, 999, 100); hipMemcpy(h3, d, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(kmul<5>, dim3(1), dim3(1), 0, 0, d, 999, 100); hipMemcpy(h4, d, 8, hipMemcpyDeviceToHost);
    printf("agree: %d %d add %d\n", h0[0] == h1[0], h0[0] == h2[0], h3[0] == h4[0]);
    return 0;
}
