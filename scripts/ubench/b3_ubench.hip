// Microbenchmark: BLAKE3 single-block compressions per second on gfx950 (independent chains)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../xfg-stark_amd/csrc/blake3.hpp"
using namespace xfg;
template <int CHAINS>
__global__ __launch_bounds__(256) void kb(Digest* out, int iters) {
    Digest d[CHAINS];
    for (int c = 0; c < CHAINS; c++)
        for (int i = 0; i < 8; i++) d[c].w[i] = threadIdx.x * 31 + i + c * 7;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) d[c] = b3_merge(d[c], d[c]);
    }
    Digest r = d[0];
    for (int c = 1; c < CHAINS; c++) for (int i = 0; i < 8; i++) r.w[i] ^= d[c].w[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
int main(int argc, char** argv) {
    Digest* d;
    const int blocks = 256 * 8, threads = 256, iters = argc > 1 ? atoi(argv[1]) : 64;
    hipMalloc(&d, (size_t)blocks * threads * sizeof(Digest));
    for (int v = 0; v < 3; v++) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        int chains = v == 0 ? 1 : (v == 1 ? 2 : 4);
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            if (v == 0) hipLaunchKernelGGL(kb<1>, dim3(blocks), dim3(threads), 0, 0, d, iters);
            if (v == 1) hipLaunchKernelGGL(kb<2>, dim3(blocks), dim3(threads), 0, 0, d, iters);
            if (v == 2) hipLaunchKernelGGL(kb<4>, dim3(blocks), dim3(threads), 0, 0, d, iters);
            hipEventRecord(b); hipEventSynchronize(b);
        }
        float ms; hipEventElapsedTime(&ms, a, b);
        double comps = (double)blocks * threads * iters * chains;
        printf("chains=%d: %.3f ms  %.1f G compressions/s  (%.1f T lane-instr/s at 686/comp)\n", chains, ms,
               comps / ms / 1e6, comps * 686 / ms / 1e9);
    }
    return 0;
}
