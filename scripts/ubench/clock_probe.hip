// In-kernel shader clock while the prover's kernels run (MI355X_MICROARCH.md "DVFS give-back" (6)):
// a one-wave probe on its own stream stamps s_memtime (shader cycles) and s_memrealtime (100 MHz)
// around a sleep loop that lasts as long as the measured work; clock = dcycles / dreal * 100 MHz.
// Build: hipcc -O2 --offload-arch=gfx950 -I include -o clock_probe scripts/ubench/clock_probe.hip \
//        -L xfg-stark_amd -lxfgstark -Wl,-rpath,$PWD/xfg-stark_amd
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "xfg_stark.h"

__global__ void probe(unsigned long long* out, unsigned long long ticks) {
    if (threadIdx.x) return;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r = r0;
    while (r - r0 < ticks) {
        __builtin_amdgcn_s_sleep(127);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[0] = t1 - t0;
    out[1] = r - r0;
}

static double run_probe(hipStream_t s, unsigned long long* d, double seconds, void (*work)(void*), void* arg) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, s, d, (unsigned long long)(seconds * 1e8));
    if (work) work(arg);
    unsigned long long h[2];
    hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    return (double)h[0] / (double)h[1] * 100.0;  // MHz
}

struct LdeArg {
    xfg_ctx* c;
    int iters;
    double ms;
};
static void lde_work(void* p) {
    LdeArg* a = (LdeArg*)p;
    if (xfg_bench_lde(a->c, 64, 1 << 16, 8, a->iters, &a->ms) != 0) { printf("bench_lde failed\n"); exit(1); }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 400;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned long long* d;
    hipMalloc(&d, 16);
    printf("idle: %.0f MHz\n", run_probe(s, d, 0.2, nullptr, nullptr));
    xfg_ctx* c = xfg_ctx_create(0);
    if (!c) { printf("no ctx\n"); return 1; }
    LdeArg a{c, 20, 0};
    lde_work(&a);  // warm + time
    a.iters = iters;
    const double sec = a.ms * iters * 1e-3;
    const double mhz = run_probe(s, d, sec * 0.9, lde_work, &a);
    printf("trace LDE (64 proofs x 7 cols, n=2^16, beta 8): %.4f ms per launch set, in-kernel clock %.0f MHz\n", a.ms, mhz);
    xfg_ctx_destroy(c);
    return 0;
}
