// Microbenchmark: HBM copy bandwidth on gfx950 by access width per lane (8 B vs 16 B), and a
// strided-row pattern like the NTT passes (each wave instruction touching 128 B segments)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned long long u64;
__global__ void copy8(const u64* __restrict__ a, u64* __restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void copy16(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, size_t n2) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
// 16 lanes per 128 B row segment: lane l of a wave -> row (l >> 4), word (l & 15); rows 4 KB apart
__global__ void copy8_seg(const u64* __restrict__ a, u64* __restrict__ b, size_t n) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < n; i += nthreads) {
        // permute index: within each 4096-element tile, element e -> (e & 15) + ((e >> 4) & 255) * 16 ... same set, 128 B runs
        const size_t t = i & ~(size_t)4095, e = i & 4095;
        const size_t j = t + ((e & 15) | ((e >> 4) << 4));
        b[j] = a[j];
    }
}
int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 8;
    u64 *a, *b;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {1024, 4096, 16384}) {
        for (int v = 0; v < 3; v++) {
            float best = 1e9;
            for (int rep = 0; rep < 5; rep++) {
                hipEventRecord(e0);
                if (v == 0) hipLaunchKernelGGL(copy8, dim3(grid), dim3(256), 0, 0, a, b, n);
                if (v == 1) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, (const ulonglong2*)a, (ulonglong2*)b, n / 2);
                if (v == 2) hipLaunchKernelGGL(copy8_seg, dim3(grid), dim3(256), 0, 0, a, b, n);
                hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("grid %5d %-9s %.3f ms  %.2f TB/s (read+write)\n", grid, v == 0 ? "8B" : v == 1 ? "16B" : "8B-seg", best,
                   2.0 * bytes / best / 1e9);
        }
    }
    return 0;
}
