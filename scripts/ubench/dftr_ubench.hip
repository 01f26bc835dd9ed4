// Per-element cost of the in-register Goldilocks DFTs dft_reg<LOGR> for radix 16, 32 and 64
// (twiddles inside all three are powers of two: w_32 = 2^78, w_64 = 2^39), and of the general
// multiply. Prints G element-levels/s (elements x log2 R per second) and a checksum per kernel; the
// checksum of each DFT is compared against a host DFT of the first thread's vector.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNTT_SRC='"../../xfg-stark_amd/csrc/ntt.hip"' dftr_ubench.hip
#include NTT_SRC
#include <stdio.h>
namespace xfg {
template <int LOGR>
__global__ __launch_bounds__(256) void k_dft(u64* io, int iters) {
    constexpr int R = 1 << LOGR;
    u64 v[R];
    const size_t base = (size_t)blockIdx.x * 256 * R + threadIdx.x;
    for (int i = 0; i < R; i++) v[i] = io[base + 256 * i];
    for (int it = 0; it < iters; it++) {
        dft_reg<LOGR, false>(v);
#pragma unroll
        for (int i = 0; i < R; i++) v[i] = canon(v[i]);
    }
    for (int i = 0; i < R; i++) io[base + 256 * i] = v[i];
}
}  // namespace xfg
using namespace xfg;
static u64 hmul(u64 a, u64 b) { return (u64)(((unsigned __int128)a * b) % P); }
static u64 hpow(u64 b, u64 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r = hmul(r, b);
        b = hmul(b, b);
        e >>= 1;
    }
    return r;
}
template <int LOGR>
static void run(u64* d, const u64* h, size_t cnt, int blocks) {
    constexpr int R = 1 << LOGR;
    const int iters = 32;
    (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_dft<LOGR>, dim3(blocks), dim3(256), 0, 0, d, 1);
    // correctness: thread 0 of block 0 after one DFT
    u64 out[64];
    for (int i = 0; i < R; i++) (void)hipMemcpy(&out[i], d + 256 * i, 8, hipMemcpyDeviceToHost);
    const u64 w = hpow(TWO_ADIC_ROOT, 1ULL << (32 - LOGR));
    int bad = 0;
    for (int q = 0; q < R; q++) {
        u64 s = 0;
        for (int r = 0; r < R; r++) s = (u64)(((unsigned __int128)s + hmul(h[256 * r], hpow(w, (u64)r * q))) % P);
        bad += s != out[q];
    }
    (void)hipMemcpy(d, h, cnt * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_dft<LOGR>, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double el = (double)blocks * 256 * R * iters * LOGR;
    printf("dft%-3d %8.3f ms  %7.2f G elem-levels/s  %s\n", R, ms, el / ms / 1e6, bad ? "MISMATCH" : "ok");
}
int main() {
    const int blocks = 256 * 8;
    const size_t cnt = (size_t)blocks * 256 * 64;
    u64* h = (u64*)malloc(cnt * 8);
    u64 s = 0x9E3779B97F4A7C15ULL;
    for (size_t i = 0; i < cnt; i++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        h[i] = s % P;
    }
    u64* d;
    (void)hipMalloc(&d, cnt * 8);
    run<4>(d, h, cnt, blocks * 4);
    run<5>(d, h, cnt, blocks * 2);
    run<6>(d, h, cnt, blocks);
    return 0;
}
