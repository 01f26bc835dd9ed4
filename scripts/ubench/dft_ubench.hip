// Throughput + agreement of the in-register radix-16 Goldilocks DFT (dft_reg<4>) and the field
// multiply as built from NTT_SRC (-DNTT_SRC=...): prints G elements/s and a checksum of canonical
// outputs. "dft16@4w" runs the same loop with a 36 KiB dynamic LDS allocation per block, which caps
// residency at 4 blocks per CU (4 waves per SIMD) like the LDS-bound NTT passes.
#include NTT_SRC
#include <stdio.h>
namespace xfg {
__global__ __launch_bounds__(256) void k_dft_loop(u64* io, int iters) {
    u64 v[16];
    for (int i = 0; i < 16; i++) v[i] = io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i];
    for (int it = 0; it < iters; it++) {
        dft_reg<4, false>(v);
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = canon(v[i]);
    }
    for (int i = 0; i < 16; i++) io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i] = v[i];
}
__global__ __launch_bounds__(256) void k_dft_loop_lds(u64* io, int iters) {
    extern __shared__ u64 sh[];
    u64 v[16];
    for (int i = 0; i < 16; i++) v[i] = io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i];
    for (int it = 0; it < iters; it++) {
        dft_reg<4, false>(v);
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = canon(v[i]);
    }
    sh[threadIdx.x] = v[0];
    __syncthreads();
    v[0] = sh[threadIdx.x];
    for (int i = 0; i < 16; i++) io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i] = v[i];
}
__global__ __launch_bounds__(256) void k_mul_loop(u64* io, int iters) {
    u64 v[16], w[16];
    for (int i = 0; i < 16; i++) { v[i] = io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i]; w[i] = v[i] ^ 0x1234567ULL; w[i] = w[i] % P; }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = gl_mul(v[i], w[i]);
    }
    for (int i = 0; i < 16; i++) io[(size_t)blockIdx.x * 4096 + threadIdx.x + 256 * i] = v[i];
}
}
using namespace xfg;
int main() {
    const int blocks = 256 * 16, iters = 64;
    const size_t cnt = (size_t)blocks * 4096;
    u64* h = (u64*)malloc(cnt * 8);
    u64 s = 0x9E3779B97F4A7C15ULL;
    for (size_t i = 0; i < cnt; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = s % P; }
    u64* d;
    (void)hipMalloc(&d, cnt * 8);
    struct { const char* n; void (*f)(u64*, int); double per; size_t lds; } ks[] = {
        {"dft16", k_dft_loop, 16.0, 0}, {"dft16@4w", k_dft_loop_lds, 16.0, 36 * 1024}, {"mul", k_mul_loop, 16.0, 0}};
    for (auto& k : ks) {
        (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), k.lds, 0, d, 1);
        (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), k.lds, 0, d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        u64* o = (u64*)malloc(cnt * 8);
        (void)hipMemcpy(o, d, cnt * 8, hipMemcpyDeviceToHost);
        u64 sum = 0;
        for (size_t i = 0; i < cnt; i++) sum = sum * 31 + (o[i] % P);
        free(o);
        const double elems = (double)blocks * 256 * iters * k.per;
        printf("%-9s %8.3f ms  %7.2f G elem-ops/s  checksum %016llx\n", k.n, ms, elems / ms / 1e6, (unsigned long long)sum);
    }
    return 0;
}
