// Microbenchmark: the HBM copy rate gfx950 sustains, and the memory skeleton of the 2^16 LDE's pass B.
//
// (1) plain copies of 2 GiB (read + write bytes counted): 8 or 16 bytes per lane, U loads in flight per
//     lane before the U stores (unrolled grid-stride loop), plain or nontemporal, grids of 1-16 blocks per
//     CU; each variant timed over 20 back-to-back launches after 3 warm ones (the clock settles only under
//     sustained load, profiles/r04/lde_ramp.txt), best of 3 windows.
// (2) pass-B-shaped copies, the trace LDE's intermediate (64 proofs x 7 columns x 8 cosets of 2^16 words)
//     read and the same bytes written as the LDE: 256-thread blocks of 16 rows x 256 words, every thread
//     16 loads in flight and then 16 stores, as ntt_pass_b_tq's loads and stores move them
//       rowmajor8  -- the intermediate as [k1][j2] rows of 2 KB, 8 B per lane, lanes along a row (4 rows x
//                     128 B per wave instruction): what pass B reads today
//       tile8      -- tile-major [tile][j2][16 rows]: lanes down the 16 rows of a column first (512
//                     contiguous bytes per wave instruction)
//       tile16     -- tile-major, 16 B per lane (two rows of a column per lane; 1 KiB per instruction, 8
//                     loads per thread)
//     and the stores of all three as pass B stores the LDE (16 consecutive rows of an output column = 128 B
//     per segment, 4 segments per instruction).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy16(const u64x2* __restrict__ a, u64x2* __restrict__ b, size_t n2) {
    const size_t T = (size_t)gridDim.x * 256;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n2; i0 += T * U) {
        u64x2 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = i0 + (size_t)u * 256;
            v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = i0 + (size_t)u * 256;
            if (NT) __builtin_nontemporal_store(v[u], b + i);
            else b[i] = v[u];
        }
    }
}
template <int U>
__global__ __launch_bounds__(256) void copy8(const u64* __restrict__ a, u64* __restrict__ b, size_t n) {
    const size_t T = (size_t)gridDim.x * 256;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += T * U) {
        u64 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = a[i0 + (size_t)u * 256];
#pragma unroll
        for (int u = 0; u < U; u++) b[i0 + (size_t)u * 256] = v[u];
    }
}

// read-only (sum of the words, one store per thread) and write-only (fill) streams of the same shape
template <int U>
__global__ __launch_bounds__(256) void read16(const u64x2* __restrict__ a, u64* __restrict__ sink, size_t n2) {
    const size_t T = (size_t)gridDim.x * 256;
    u64 acc = 0;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n2; i0 += T * U) {
        u64x2 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = a[i0 + (size_t)u * 256];
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u][0] ^ v[u][1];
    }
    if (acc == 0x123456789ULL) sink[0] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void write16(u64x2* __restrict__ b, size_t n2) {
    const size_t T = (size_t)gridDim.x * 256;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n2; i0 += T * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = i0 + (size_t)u * 256;
            b[i] = u64x2{i, i + 1};
        }
    }
}

// pass-B shapes: one block per (16-row tile, plane); plane = 2^16 words as [256 rows][256 cols]
template <int MODE>
__global__ __launch_bounds__(256) void passb(const u64* __restrict__ y, u64* __restrict__ out) {
    const int tile = blockIdx.x, plane = blockIdx.y, tid = threadIdx.x;
    const u64* yp = y + ((size_t)plane << 16);
    u64* op = out + ((size_t)plane << 16) + tile * 16;
    u64 v[16];
    if (MODE == 0) {  // row-major, lanes along a row: seq0 = tid / 16, j0 = tid % 16, elements j0 + 16 r
        const int seq0 = tid >> 4, j0 = tid & 15;
        const u64* p = yp + ((size_t)(tile * 16 + seq0) << 8) + j0;
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = p[r * 16];
    } else if (MODE == 1) {  // tile-major [tile][col][16]: lanes down a column's 16 rows, col = j0 + 16 r
        const int seq0 = tid & 15, j0 = tid >> 4;
        const u64* p = yp + ((size_t)tile << 12) + j0 * 16 + seq0;
#pragma unroll
        for (int r = 0; r < 16; r++) v[r] = p[r * 256];
    } else {  // tile-major, 16 B per lane: lane pairs cover 4 rows; 8 loads of (row, row + 1) per thread
        const int pr = tid & 7, j0 = tid >> 3;  // rows 2 pr, 2 pr + 1 of columns j0 + 32 r
        const u64x2* p = reinterpret_cast<const u64x2*>(yp + ((size_t)tile << 12) + j0 * 16 + 2 * pr);
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u64x2 w = p[r * 256];
            v[2 * r] = w[0];
            v[2 * r + 1] = w[1];
        }
    }
    // stores as pass B's second step: lane -> (seq = g & 15, j = g >> 4), outputs (j + 16 r) * 256 + seq
    const int seq = tid & 15, j = tid >> 4;
#pragma unroll
    for (int r = 0; r < 16; r++) op[((size_t)(j + 16 * r) << 8) + seq] = v[r] ^ (u64)r;
}

static hipEvent_t e0, e1;
template <class F>
static float window(F launch, int iters = 20) {
    float best = 1e30f;
    for (int w = 0; w < 3; w++) {
        for (int i = 0; i < 3; i++) launch();
        hipEventRecord(e0);
        for (int i = 0; i < iters; i++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms / iters < best) best = ms / iters;
    }
    return best;
}

int main() {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t bytes = (size_t)2 << 30, n = bytes / 8;
    u64 *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("# plain copies, 2 GiB, read + write bytes, ms per launch (20-launch windows, best of 3); %d CUs\n", cus);
    for (int per : {1, 2, 4, 8, 16}) {
        const int grid = cus * per;
        struct V { const char* name; float ms; };
        std::vector<V> vs;
        vs.push_back({"8B u1", window([&] { hipLaunchKernelGGL((copy8<1>), dim3(grid), dim3(256), 0, 0, a, b, n); })});
        vs.push_back({"8B u8", window([&] { hipLaunchKernelGGL((copy8<8>), dim3(grid), dim3(256), 0, 0, a, b, n); })});
        vs.push_back({"16B u1", window([&] { hipLaunchKernelGGL((copy16<1, false>), dim3(grid), dim3(256), 0, 0, (const u64x2*)a, (u64x2*)b, n / 2); })});
        vs.push_back({"16B u4", window([&] { hipLaunchKernelGGL((copy16<4, false>), dim3(grid), dim3(256), 0, 0, (const u64x2*)a, (u64x2*)b, n / 2); })});
        vs.push_back({"16B u8", window([&] { hipLaunchKernelGGL((copy16<8, false>), dim3(grid), dim3(256), 0, 0, (const u64x2*)a, (u64x2*)b, n / 2); })});
        vs.push_back({"16B u4 nt", window([&] { hipLaunchKernelGGL((copy16<4, true>), dim3(grid), dim3(256), 0, 0, (const u64x2*)a, (u64x2*)b, n / 2); })});
        for (auto& v : vs) printf("blocks/CU %2d  %-10s %.3f ms  %.2f TB/s\n", per, v.name, v.ms, 2.0 * bytes / v.ms / 1e9);
    }
    printf("# one direction only (bytes moved = 2 GiB)\n");
    for (int per : {1, 2, 4, 8}) {
        const int grid = cus * per;
        const float r = window([&] { hipLaunchKernelGGL((read16<8>), dim3(grid), dim3(256), 0, 0, (const u64x2*)a, b, n / 2); });
        const float w = window([&] { hipLaunchKernelGGL((write16<8>), dim3(grid), dim3(256), 0, 0, (u64x2*)b, n / 2); });
        printf("blocks/CU %2d  read 16B u8 %.3f ms %.2f TB/s   write 16B u8 %.3f ms %.2f TB/s\n", per, r, bytes / r / 1e9, w,
               bytes / w / 1e9);
    }
    // pass B shape: 64 proofs x 7 columns x 8 cosets = 3584 planes of 2^16 words = 1.84 GB each way
    const int planes = 3584;
    const size_t pb = (size_t)planes << 19;  // bytes
    u64 *y, *o;
    hipMalloc(&y, pb);
    hipMalloc(&o, pb);
    hipMemset(y, 2, pb);
    printf("# pass-B-shaped copies: %d planes of 2^16 words (%.2f GB read + %.2f GB written), 16 x 256 tiles\n", planes,
           pb / 1e9, pb / 1e9);
    const char* names[3] = {"rowmajor8", "tile8", "tile16"};
    for (int m = 0; m < 3; m++) {
        const float ms = window([&] {
            if (m == 0) hipLaunchKernelGGL(passb<0>, dim3(16, planes), dim3(256), 0, 0, y, o);
            if (m == 1) hipLaunchKernelGGL(passb<1>, dim3(16, planes), dim3(256), 0, 0, y, o);
            if (m == 2) hipLaunchKernelGGL(passb<2>, dim3(16, planes), dim3(256), 0, 0, y, o);
        }, 10);
        printf("%-10s %.3f ms  %.2f TB/s\n", names[m], ms, 2.0 * pb / ms / 1e9);
    }
    return 0;
}
