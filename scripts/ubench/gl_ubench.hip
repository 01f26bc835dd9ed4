// Microbenchmark + correctness: Goldilocks add / sub / mul formulations on gfx950.
// C forms (gl.hpp) vs carry-flag inline-asm forms (v_*_co_u32 chains through VCC).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../xfg-stark_amd/csrc/gl.hpp"
using namespace xfg;

__device__ __forceinline__ u64 add_asm(u64 a, u64 b) {
    // q = p - b; d = a - q (borrow -> a + b < p); r = borrow ? d - EPS : d
    u32 al = (u32)a, ah = (u32)(a >> 32), bl = (u32)b, bh = (u32)(b >> 32), ql, qh, dl, dh, e;
    asm volatile(
        "v_sub_co_u32_e32 %0, vcc, 1, %7\n\t"
        "v_subb_co_u32_e32 %1, vcc, -1, %8, vcc\n\t"
        "v_sub_co_u32_e32 %2, vcc, %5, %0\n\t"
        "v_subb_co_u32_e32 %3, vcc, %6, %1, vcc\n\t"
        "v_cndmask_b32_e64 %4, 0, -1, vcc\n\t"
        "v_sub_co_u32_e32 %2, vcc, %2, %4\n\t"
        "v_subbrev_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
        : "=&v"(ql), "=&v"(qh), "=&v"(dl), "=&v"(dh), "=&v"(e)
        : "v"(al), "v"(ah), "v"(bl), "v"(bh)
        : "vcc");
    return (u64)dl | ((u64)dh << 32);
}
// carries in compiler-allocated SGPR pairs (not VCC), so independent adds can interleave
__device__ __forceinline__ u64 add_sg(u64 a, u64 b) {
    u32 al = (u32)a, ah = (u32)(a >> 32), bl = (u32)b, bh = (u32)(b >> 32), ql, qh, dl, dh, e;
    u64 c0, c1, c2, c3;
    asm volatile(
        "v_sub_co_u32_e64 %[ql], %[c0], 1, %[bl]\n\t"
        "v_subb_co_u32_e64 %[qh], %[c1], -1, %[bh], %[c0]\n\t"
        "v_sub_co_u32_e64 %[dl], %[c2], %[al], %[ql]\n\t"
        "v_subb_co_u32_e64 %[dh], %[c3], %[ah], %[qh], %[c2]\n\t"
        "v_cndmask_b32_e64 %[e], 0, -1, %[c3]\n\t"
        : [ql] "=&v"(ql), [qh] "=&v"(qh), [dl] "=&v"(dl), [dh] "=&v"(dh), [e] "=&v"(e), [c0] "=&s"(c0),
          [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3)
        : [al] "v"(al), [ah] "v"(ah), [bl] "v"(bl), [bh] "v"(bh));
    u64 d = (u64)dl | ((u64)dh << 32);
    return d - (u64)e;  // borrowed: a + b = d - EPS (mod 2^64); e = EPS or 0
}
__device__ __forceinline__ u64 sub_sg(u64 a, u64 b) {
    u32 al = (u32)a, ah = (u32)(a >> 32), bl = (u32)b, bh = (u32)(b >> 32), dl, dh, e;
    u64 c0, c1;
    asm volatile(
        "v_sub_co_u32_e64 %[dl], %[c0], %[al], %[bl]\n\t"
        "v_subb_co_u32_e64 %[dh], %[c1], %[ah], %[bh], %[c0]\n\t"
        "v_cndmask_b32_e64 %[e], 0, -1, %[c1]\n\t"
        : [dl] "=&v"(dl), [dh] "=&v"(dh), [e] "=&v"(e), [c0] "=&s"(c0), [c1] "=&s"(c1)
        : [al] "v"(al), [ah] "v"(ah), [bl] "v"(bl), [bh] "v"(bh));
    u64 d = (u64)dl | ((u64)dh << 32);
    return d - (u64)e;
}
__device__ __forceinline__ u64 sub_asm(u64 a, u64 b) {
    u32 al = (u32)a, ah = (u32)(a >> 32), bl = (u32)b, bh = (u32)(b >> 32), dl, dh, e;
    asm volatile(
        "v_sub_co_u32_e32 %0, vcc, %3, %5\n\t"
        "v_subb_co_u32_e32 %1, vcc, %4, %6, vcc\n\t"
        "v_cndmask_b32_e64 %2, 0, -1, vcc\n\t"
        "v_sub_co_u32_e32 %0, vcc, %0, %2\n\t"
        "v_subbrev_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        : "=&v"(dl), "=&v"(dh), "=&v"(e)
        : "v"(al), "v"(ah), "v"(bl), "v"(bh)
        : "vcc");
    return (u64)dl | ((u64)dh << 32);
}
// reduce hi * 2^64 + lo (canonical result) with carry-flag chains
__device__ __forceinline__ u64 reduce_asm(u64 hi, u64 lo) {
    u32 ll = (u32)lo, lh = (u32)(lo >> 32), hl = (u32)hi, hh = (u32)(hi >> 32);
    u32 t0l, t0h, t1l, t1h, e, ul, uh;
    asm volatile(
        // t0 = lo - hh; borrow -> t0 -= EPS
        "v_sub_co_u32_e32 %0, vcc, %9, %12\n\t"
        "v_subbrev_co_u32_e32 %1, vcc, 0, %10, vcc\n\t"
        "v_cndmask_b32_e64 %4, 0, -1, vcc\n\t"
        "v_sub_co_u32_e32 %0, vcc, %0, %4\n\t"
        "v_subbrev_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        // t1 = hl * EPS = (hl << 32) - hl
        "v_sub_co_u32_e32 %2, vcc, 0, %11\n\t"
        "v_subbrev_co_u32_e32 %3, vcc, 0, %11, vcc\n\t"
        // t2 = t0 + t1; carry -> += EPS
        "v_add_co_u32_e32 %0, vcc, %0, %2\n\t"
        "v_addc_co_u32_e32 %1, vcc, %1, %3, vcc\n\t"
        "v_cndmask_b32_e64 %4, 0, -1, vcc\n\t"
        "v_add_co_u32_e32 %0, vcc, %0, %4\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        // canonical: u = t2 + EPS carries iff t2 >= p
        "v_add_co_u32_e32 %5, vcc, -1, %0\n\t"
        "v_addc_co_u32_e32 %6, vcc, 0, %1, vcc\n\t"
        "v_cndmask_b32_e32 %0, %0, %5, vcc\n\t"
        "v_cndmask_b32_e32 %1, %1, %6, vcc\n\t"
        : "=&v"(t0l), "=&v"(t0h), "=&v"(t1l), "=&v"(t1h), "=&v"(e), "=&v"(ul), "=&v"(uh)
        : "v"(0), "v"(0), "v"(ll), "v"(lh), "v"(hl), "v"(hh)
        : "vcc");
    return (u64)t0l | ((u64)t0h << 32);
}
__device__ __forceinline__ u64 mul_asm(u64 a, u64 b) {
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = (u64)a0 * b0;
    const u64 t1 = (u64)a0 * b1 + (p00 >> 32);
    const u64 t2 = (u64)a1 * b0 + (u32)t1;
    const u64 lo = (u64)(u32)p00 | ((u64)(u32)t2 << 32);
    const u64 hi = (u64)a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    return reduce_asm(hi, lo);
}

// C forms with the carries taken from __builtin_*_overflow (the compiler keeps them in SGPR pairs)
__device__ __forceinline__ u64 add_v6(u64 a, u64 b) {
    // a, b < p: s = a + b; s >= p iff carry or s + EPS carries
    u64 s, t;
    const bool c1 = __builtin_add_overflow(a, b, &s);
    const bool c2 = __builtin_add_overflow(s, EPS, &t);
    return (c1 | c2) ? t : s;
}
__device__ __forceinline__ u64 sub_v5(u64 a, u64 b) {
    u64 d;
    const bool c = __builtin_sub_overflow(a, b, &d);
    return c ? d - EPS : d;
}
__device__ __forceinline__ u64 reduce_v(u64 hi, u64 lo) {
    const u64 hh = hi >> 32, hl = hi & EPS;
    u64 t0, t2, u;
    const bool b = __builtin_sub_overflow(lo, hh, &t0);
    t0 = b ? t0 - EPS : t0;
    const u64 t1 = (hl << 32) - hl;
    const bool c = __builtin_add_overflow(t0, t1, &t2);
    const bool c2 = __builtin_add_overflow(t2, EPS, &u);
    return (c | c2) ? u : t2;
}
__device__ __forceinline__ u64 mul_v(u64 a, u64 b) {
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = (u64)a0 * b0;
    const u64 t1 = (u64)a0 * b1 + (p00 >> 32);
    const u64 t2 = (u64)a1 * b0 + (u32)t1;
    const u64 lo = (u64)(u32)p00 | ((u64)(u32)t2 << 32);
    const u64 hi = (u64)a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    return reduce_v(hi, lo);
}

#define KERNEL(NAME, OP)                                                                      \
    __global__ __launch_bounds__(256) void NAME(const u64* in, u64* out, int iters) {         \
        size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;                              \
        u64 x[8];                                                                             \
        for (int c = 0; c < 8; c++) x[c] = in[(g * 8 + c) & 65535];                          \
        u64 y = in[(g + 12345) & 65535];                                                      \
        for (int it = 0; it < iters; it++) {                                                  \
            _Pragma("unroll") for (int c = 0; c < 8; c++) x[c] = OP(x[c], y);                 \
        }                                                                                     \
        u64 r = 0;                                                                            \
        for (int c = 0; c < 8; c++) r ^= x[c];                                                \
        out[g] = r;                                                                           \
    }                                                                                         \
    __global__ void NAME##_one(const u64* a, const u64* b, u64* o, int n) {                  \
        int i = blockIdx.x * blockDim.x + threadIdx.x;                                        \
        if (i < n) o[i] = OP(a[i], b[i]);                                                     \
    }
KERNEL(k_add_c, gl_add)
KERNEL(k_add_asm, add_asm)
KERNEL(k_sub_c, gl_sub)
KERNEL(k_sub_asm, sub_asm)
KERNEL(k_mul_c, gl_mul)
KERNEL(k_add_sg, add_sg)
KERNEL(k_sub_sg, sub_sg)
KERNEL(k_mul_asm, mul_asm)
KERNEL(k_add_v6, add_v6)
KERNEL(k_sub_v5, sub_v5)
KERNEL(k_mul_v, mul_v)

static u64 rnd(u64& s) {
    s += 0x9E3779B97F4A7C15ULL;
    u64 z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
int main() {
    const int N = 1 << 20;
    u64 *ha = (u64*)malloc(N * 8), *hb = (u64*)malloc(N * 8), *ho = (u64*)malloc(N * 8);
    u64 s = 1;
    for (int i = 0; i < N; i++) {
        ha[i] = rnd(s) % P;
        hb[i] = rnd(s) % P;
    }
    // edge values
    u64 edge[] = {0, 1, 2, EPS, EPS + 1, P - 1, P - 2, P - EPS, 1ULL << 32, (1ULL << 63), P - (1ULL << 32)};
    int ne = sizeof edge / 8, k = 0;
    for (int i = 0; i < ne; i++)
        for (int j = 0; j < ne; j++, k++) {
            ha[k] = edge[i];
            hb[k] = edge[j];
        }
    u64 *da, *db, *dout, *dbig;
    hipMalloc(&da, N * 8);
    hipMalloc(&db, N * 8);
    hipMalloc(&dout, N * 8);
    hipMalloc(&dbig, (size_t)256 * 8 * 256 * 8);
    hipMemcpy(da, ha, N * 8, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, N * 8, hipMemcpyHostToDevice);
    struct K {
        const char* n;
        void (*f)(const u64*, u64*, int);
        void (*one)(const u64*, const u64*, u64*, int);
        int kind;
    } ks[] = {{"add C", k_add_c, k_add_c_one, 0},   {"add asm", k_add_asm, k_add_asm_one, 0},
              {"sub C", k_sub_c, k_sub_c_one, 1},   {"sub asm", k_sub_asm, k_sub_asm_one, 1},
              {"mul C", k_mul_c, k_mul_c_one, 2},   {"mul asm", k_mul_asm, k_mul_asm_one, 2},
              {"add sg", k_add_sg, k_add_sg_one, 0}, {"sub sg", k_sub_sg, k_sub_sg_one, 1},
              {"add v6", k_add_v6, k_add_v6_one, 0}, {"sub v5", k_sub_v5, k_sub_v5_one, 1},
              {"mul v", k_mul_v, k_mul_v_one, 2}};
    for (auto& kk : ks) {
        hipLaunchKernelGGL(kk.one, dim3(N / 256), dim3(256), 0, 0, da, db, dout, N);
        hipMemcpy(ho, dout, N * 8, hipMemcpyDeviceToHost);
        long bad = 0;
        for (int i = 0; i < N; i++) {
            u64 e = kk.kind == 0 ? gl_add(ha[i], hb[i]) : kk.kind == 1 ? gl_sub(ha[i], hb[i]) : gl_mul(ha[i], hb[i]);
            if (e != ho[i]) bad++;
        }
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float ms = 0;
        const int blocks = 256 * 8, iters = kk.kind == 2 ? 64 : 256;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kk.f, dim3(blocks), dim3(256), 0, 0, da, dbig, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        double ops = (double)blocks * 256 * iters * 8;
        printf("%-8s mismatches %ld / %d   %.3f ms  %.2f T ops/s\n", kk.n, bad, N, ms, ops / ms / 1e9);
    }
    return 0;
}
