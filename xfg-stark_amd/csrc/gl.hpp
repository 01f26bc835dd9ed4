// Goldilocks field p = 2^64 - 2^32 + 1 for CDNA4 (gfx950) kernels and the host orchestration.
// Same field as Winterfell `math::fields::f64::BaseElement` used by the reference AIR
// (reference src/burn_mint_air.rs:17). All values held in HBM are canonical (< p), so the proof
// bytes are simply little-endian u64 words.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xfg {

typedef uint64_t u64;
typedef uint32_t u32;

constexpr u64 P = 0xFFFFFFFF00000001ULL;
constexpr u64 EPS = 0xFFFFFFFFULL;  // 2^64 mod p
constexpr u64 GEN = 7;              // multiplicative generator == Winterfell domain offset
constexpr u64 TWO_ADIC_ROOT = 1753635133440165772ULL;  // 7^((p-1)/2^32)

__host__ __device__ __forceinline__ u64 gl_add(u64 a, u64 b) {
    // a + b == a - (p - b); the borrow case adds p back, i.e. subtracts EPS mod 2^64
    // (measured on gfx950: 6.0 T/s vs 4.2 T/s for the carry + compare form)
    u64 q = P - b;
    u64 d = a - q;
    return (a < q) ? d - EPS : d;
}
__host__ __device__ __forceinline__ u64 gl_sub(u64 a, u64 b) {
    u64 d = a - b;
    return (a < b) ? d - EPS : d;  // borrowed: -2^64 == -EPS
}
__host__ __device__ __forceinline__ u64 gl_neg(u64 a) { return a ? P - a : 0; }

__host__ __device__ __forceinline__ u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}
// lo + t mod p for any lo and t <= (2^32 - 1)^2 (so lo + t - 2^64 + EPS < p): the carry or a carry
// of the canonicalising + EPS selects the reduced value; canonical result
__host__ __device__ __forceinline__ u64 gl_add_small(u64 lo, u64 t) {
    u64 s, u;
    const bool c = __builtin_add_overflow(lo, t, &s);
    const bool c2 = __builtin_add_overflow(s, EPS, &u);
    return (c | c2) ? u : s;
}
// reduce hi*2^64 + lo using 2^64 == 2^32 - 1 and 2^96 == -1; canonical result for any hi, lo
// (17% more multiplies/s on gfx950 than a compare-based form: scripts/ubench/gl_ubench.hip "mul v")
__host__ __device__ __forceinline__ u64 gl_reduce(u64 hi, u64 lo) {
    const u64 hh = hi >> 32, hl = hi & EPS;
    u64 t0;
    const bool b = __builtin_sub_overflow(lo, hh, &t0);
    t0 = b ? t0 - EPS : t0;  // borrowed: + p == - EPS (mod 2^64), cannot wrap since t0 >= 2^64 - 2^32
    return gl_add_small(t0, (hl << 32) - hl);
}
__host__ __device__ __forceinline__ u64 gl_mul(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    // 64x64 -> 128 product from four 32x32+64 mads (v_mad_u64_u32), carries folded into the
    // addends; 22% faster on gfx950 than the compiler's lowering of a * b / __umul64hi
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u64 p00 = (u64)a0 * b0;
    const u64 t1 = (u64)a0 * b1 + (p00 >> 32);
    const u64 t2 = (u64)a1 * b0 + (u32)t1;
    const u64 lo = (u64)(u32)p00 | ((u64)(u32)t2 << 32);
    const u64 hi = (u64)a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    return gl_reduce(hi, lo);
#else
    return gl_reduce(mulhi64(a, b), a * b);
#endif
}
__host__ __device__ __forceinline__ u64 gl_sqr(u64 a) { return gl_mul(a, a); }
__host__ __device__ inline u64 gl_pow(u64 b, u64 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r = gl_mul(r, b);
        b = gl_mul(b, b);
        e >>= 1;
    }
    return r;
}
__host__ __device__ inline u64 gl_inv(u64 a) { return gl_pow(a, P - 2); }
// winter-math get_root_of_unity(k): primitive 2^k-th root
__host__ __device__ inline u64 gl_root(unsigned k) { return gl_pow(TWO_ADIC_ROOT, 1ULL << (32 - k)); }

// ---- quadratic extension E = F[phi] / (phi^2 - phi + 2) (winter-math f64 QuadExtension):
// (a0 + a1 phi)(b0 + b1 phi) = (a0 b0 - 2 a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0) phi
struct E2 {
    u64 a, b;
};
__host__ __device__ __forceinline__ E2 e2(u64 a, u64 b = 0) { return E2{a, b}; }
__host__ __device__ __forceinline__ E2 e2_add(E2 x, E2 y) { return E2{gl_add(x.a, y.a), gl_add(x.b, y.b)}; }
__host__ __device__ __forceinline__ E2 e2_sub(E2 x, E2 y) { return E2{gl_sub(x.a, y.a), gl_sub(x.b, y.b)}; }
__host__ __device__ __forceinline__ E2 e2_mulb(E2 x, u64 s) { return E2{gl_mul(x.a, s), gl_mul(x.b, s)}; }
__host__ __device__ __forceinline__ E2 e2_mul(E2 x, E2 y) {
    const u64 a0b0 = gl_mul(x.a, y.a), a1b1 = gl_mul(x.b, y.b);
    const u64 m = gl_mul(gl_add(x.a, x.b), gl_add(y.a, y.b));
    return E2{gl_sub(a0b0, gl_add(a1b1, a1b1)), gl_sub(m, a0b0)};
}
__host__ __device__ inline E2 e2_inv(E2 x) {
    // frob(x) = (a0 + a1) - a1 phi; x * frob(x) is in F
    const E2 f{gl_add(x.a, x.b), gl_neg(x.b)};
    return e2_mulb(f, gl_inv(e2_mul(x, f).a));
}
__host__ __device__ inline E2 e2_pow(E2 b, u64 e) {
    E2 r{1, 0};
    while (e) {
        if (e & 1) r = e2_mul(r, b);
        b = e2_mul(b, b);
        e >>= 1;
    }
    return r;
}
__host__ __device__ __forceinline__ bool e2_eq(E2 x, E2 y) { return x.a == y.a && x.b == y.b; }

// field element of extension degree D (1 = base, 2 = quadratic) for D-templated kernels
template <int D>
struct FE;
template <>
struct FE<1> {
    u64 a;
    __host__ __device__ __forceinline__ static FE zero() { return FE{0}; }
    __host__ __device__ __forceinline__ static FE load(const u64* p) { return FE{p[0]}; }
    __host__ __device__ __forceinline__ void store(u64* p) const { p[0] = a; }
    __host__ __device__ __forceinline__ u64 c(int) const { return a; }
};
template <>
struct FE<2> {
    u64 a, b;
    __host__ __device__ __forceinline__ static FE zero() { return FE{0, 0}; }
    __host__ __device__ __forceinline__ static FE load(const u64* p) { return FE{p[0], p[1]}; }
    __host__ __device__ __forceinline__ void store(u64* p) const { p[0] = a; p[1] = b; }
    __host__ __device__ __forceinline__ u64 c(int i) const { return i ? b : a; }
};
__host__ __device__ __forceinline__ FE<1> fe_add(FE<1> x, FE<1> y) { return FE<1>{gl_add(x.a, y.a)}; }
__host__ __device__ __forceinline__ FE<1> fe_sub(FE<1> x, FE<1> y) { return FE<1>{gl_sub(x.a, y.a)}; }
__host__ __device__ __forceinline__ FE<1> fe_mul(FE<1> x, FE<1> y) { return FE<1>{gl_mul(x.a, y.a)}; }
__host__ __device__ __forceinline__ FE<1> fe_mulb(FE<1> x, u64 s) { return FE<1>{gl_mul(x.a, s)}; }
__host__ __device__ __forceinline__ FE<2> fe_add(FE<2> x, FE<2> y) { return FE<2>{gl_add(x.a, y.a), gl_add(x.b, y.b)}; }
__host__ __device__ __forceinline__ FE<2> fe_sub(FE<2> x, FE<2> y) { return FE<2>{gl_sub(x.a, y.a), gl_sub(x.b, y.b)}; }
__host__ __device__ __forceinline__ FE<2> fe_mulb(FE<2> x, u64 s) { return FE<2>{gl_mul(x.a, s), gl_mul(x.b, s)}; }
__host__ __device__ __forceinline__ FE<2> fe_mul(FE<2> x, FE<2> y) {
    E2 r = e2_mul(E2{x.a, x.b}, E2{y.a, y.b});
    return FE<2>{r.a, r.b};
}

}  // namespace xfg
