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

__device__ __forceinline__ u64 gl_add_dev(u64 a, u64 b);
__device__ __forceinline__ u64 gl_sub_weak(u64 a, u64 b);
__host__ __device__ __forceinline__ u64 gl_add(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return gl_add_dev(a, b);
#else
    // a + b == a - (p - b); the borrow case adds p back, i.e. subtracts EPS mod 2^64
    u64 q = P - b;
    u64 d = a - q;
    return (a < q) ? d - EPS : d;
#endif
}
__host__ __device__ __forceinline__ u64 gl_sub(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return gl_sub_weak(a, b);  // canonical for canonical a, b
#else
    u64 d = a - b;
    return (a < b) ? d - EPS : d;  // borrowed: -2^64 == -EPS
#endif
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
// ---- gfx950 instruction-level forms. The VALU is the bound of every kernel of this path, so these
// are written for instruction count: v_mad_u64_u32's carry-out and 64-bit selects by a 0/1 multiple
// of EPS replace the compiler's compare-and-select lowering. Every VALU write of an SGPR mask that a
// VALU reads back inside a statement is followed by >= 2 wait states (s_nop 1), VALU -> SALU and
// SALU -> VALU mask hand-offs need none (both as the compiler itself emits them).

// canonical lo + h * EPS for any lo and h < 2^32 (4 VALU + 1 SALU): r = lo + h EPS (carry c1);
// c1 or r >= p selects r + EPS mod 2^64 (= r + 2^64 mod p when c1, r - p otherwise)
__device__ __forceinline__ u64 gl_fold(u64 lo, u32 h) {
#if defined(__HIP_DEVICE_COMPILE__)
    u64 r, out, c1, c2;
    u32 sel;
    asm("v_mad_u64_u32 %[r], %[c1], %[h], -1, %[lo]\n\t"
        "v_cmp_lt_u64_e64 %[c2], %[pm1], %[r]\n\t"
        "s_or_b64 %[c1], %[c1], %[c2]\n\t"
        "v_cndmask_b32_e64 %[sel], 0, 1, %[c1]\n\t"
        "v_mad_u64_u32 %[out], %[c2], %[sel], -1, %[r]"
        : [r] "=&v"(r), [out] "=&v"(out), [sel] "=&v"(sel), [c1] "=&s"(c1), [c2] "=&s"(c2)
        : [h] "v"(h), [lo] "v"(lo), [pm1] "s"(P - 1)
        : "scc");
    return out;
#else
    u64 r = lo + (u64)h * EPS;
    const bool c = r < lo;
    return (c || r >= P) ? r + EPS : r;
#endif
}
// canonical a + b for canonical a, b (5 VALU + 1 SALU): s = a + b (carry c1); c1 or s >= p selects
// s + EPS mod 2^64
__device__ __forceinline__ u64 gl_add_dev(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    u64 s, out, c1, c2;
    u32 sel;
    asm("v_lshl_add_u64 %[s], %[a], 0, %[b]\n\t"
        "v_cmp_lt_u64_e64 %[c1], %[s], %[b]\n\t"
        "v_cmp_lt_u64_e64 %[c2], %[pm1], %[s]\n\t"
        "s_or_b64 %[c1], %[c1], %[c2]\n\t"
        "v_cndmask_b32_e64 %[sel], 0, 1, %[c1]\n\t"
        "v_mad_u64_u32 %[out], %[c2], %[sel], -1, %[s]"
        : [s] "=&v"(s), [out] "=&v"(out), [sel] "=&v"(sel), [c1] "=&s"(c1), [c2] "=&s"(c2)
        : [a] "v"(a), [b] "v"(b), [pm1] "s"(P - 1)
        : "scc");
    return out;
#else
    u64 s = a + b;
    return (s < b || s >= P) ? s + EPS : s;
#endif
}
// canonical x for any u64 x (3 VALU)
__device__ __forceinline__ u64 gl_canon(u64 x) {
#if defined(__HIP_DEVICE_COMPILE__)
    u64 out, c;
    u32 sel;
    asm("v_cmp_lt_u64_e64 %[c], %[pm1], %[x]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[sel], 0, 1, %[c]\n\t"
        "v_mad_u64_u32 %[out], %[c], %[sel], -1, %[x]"
        : [out] "=&v"(out), [sel] "=&v"(sel), [c] "=&s"(c)
        : [x] "v"(x), [pm1] "s"(P - 1));
    return out;
#else
    return x >= P ? x - P : x;
#endif
}
// a - b as a 64-bit value with the borrow folded once: a - b + p when a < b; for b <= a + p
// (b < p or b <= a) the result is the exact representative in [0, 2^64)
__device__ __forceinline__ u64 gl_sub_weak(u64 a, u64 b) {
    u32 b0, b1, b2, b3;
    const u32 dl = __builtin_subc((u32)a, (u32)b, 0u, &b0);
    const u32 dh = __builtin_subc((u32)(a >> 32), (u32)(b >> 32), b0, &b1);
    const u32 el = __builtin_subc(dl, b1 ? 0xFFFFFFFFu : 0u, 0u, &b2);
    const u32 eh = __builtin_subc(dh, 0u, b2, &b3);
    return ((u64)eh << 32) | el;
}
// lo - h for a 32-bit h, borrow folded once (+ p): the exact representative in [0, 2^64) for any lo
// (h <= 2^32 - 1 < p). 5 VALU as one sub / subb chain (the compiler's lowering of gl_sub_weak with a
// zero high word materialises the first borrow: 6)
__device__ __forceinline__ u64 gl_sub_u32(u64 lo, u32 h) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 d0, d1, m, e0, e1;
    u64 bb, bb2;
    asm("v_sub_co_u32_e64 %[d0], %[bb], %[l0], %[h]\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32_e64 %[d1], %[bb], %[l1], 0, %[bb]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[m], 0, -1, %[bb]\n\t"
        "v_sub_co_u32_e64 %[e0], %[bb2], %[d0], %[m]\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32_e64 %[e1], %[bb2], %[d1], 0, %[bb2]"
        : [d0] "=&v"(d0), [d1] "=&v"(d1), [m] "=&v"(m), [e0] "=&v"(e0), [e1] "=&v"(e1), [bb] "=&s"(bb),
          [bb2] "=&s"(bb2)
        : [l0] "v"((u32)lo), [l1] "v"((u32)(lo >> 32)), [h] "v"(h));
    return ((u64)e1 << 32) | e0;
#else
    return gl_sub_weak(lo, h);
#endif
}
__host__ __device__ __forceinline__ u64 gl_mul(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    // a b = lo + hl 2^64 + (hh + c) 2^96 == lo - (hh + c) + hl EPS, (hh + c) <= 2^32 - 1 for any a, b
    // < 2^64 (15 VALU + 1 SALU; the round-4 product + gl_sub_weak + gl_fold was 18, the compiler's own lowering
    // of the same math 24). The product's carry c is never materialised: it is the borrow-in of the
    // subtraction lo - hh - c, done on the words of the partial products as they come out of the
    // mads (lo = (p.lo, t2.lo)), so neither the 64-bit assembly of lo nor hh + c costs an instruction;
    // a borrow out of the high word adds p (- EPS mod 2^64) once, then gl_fold adds hl EPS.
    // Each VALU-written carry / borrow mask is read by a VALU only after >= 2 wait states.
    u64 p, t1, t2, hi, x, s, c;
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    asm("v_mad_u64_u32 %[p], %[s], %[a0], %[b0], 0\n\t"
        "v_lshrrev_b64 %[x], 32, %[p]\n\t"
        "v_mad_u64_u32 %[t1], %[s], %[a0], %[b1], %[x]\n\t"
        "v_mad_u64_u32 %[t2], %[c], %[a1], %[b0], %[t1]\n\t"
        "v_lshrrev_b64 %[x], 32, %[t2]\n\t"
        "v_mad_u64_u32 %[hi], %[s], %[a1], %[b1], %[x]"
        : [p] "=&v"(p), [x] "=&v"(x), [t1] "=&v"(t1), [t2] "=&v"(t2), [hi] "=&v"(hi), [s] "=&s"(s), [c] "=&s"(c)
        : [a0] "v"(a0), [a1] "v"(a1), [b0] "v"(b0), [b1] "v"(b1));
    u32 d0, d1, m, e0, e1;
    u64 bb, bb2;
    asm("s_nop 1\n\t"
        "v_subb_co_u32_e64 %[d0], %[bb], %[l0], %[hh], %[c]\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32_e64 %[d1], %[bb], %[l1], 0, %[bb]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[m], 0, -1, %[bb]\n\t"
        "v_sub_co_u32_e64 %[e0], %[bb2], %[d0], %[m]\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32_e64 %[e1], %[bb2], %[d1], 0, %[bb2]"
        : [d0] "=&v"(d0), [d1] "=&v"(d1), [m] "=&v"(m), [e0] "=&v"(e0), [e1] "=&v"(e1), [bb] "=&s"(bb),
          [bb2] "=&s"(bb2)
        : [l0] "v"((u32)p), [l1] "v"((u32)t2), [hh] "v"((u32)(hi >> 32)), [c] "s"(c));
    return gl_fold(((u64)e1 << 32) | e0, (u32)hi);
#else
    return gl_reduce(mulhi64(a, b), a * b);
#endif
}
// two independent products a * b, c * d with their instruction streams interleaved: each one's
// carry / borrow wait states are filled by the other's instructions (3 s_nop 0 for the pair instead of
// 4 s_nop 1 each); results identical to gl_mul
__host__ __device__ __forceinline__ void gl_mul2(u64& a, u64 b, u64& c, u64 d) {
#if defined(__HIP_DEVICE_COMPILE__)
    u64 pA, t1A, t2A, hiA, xA, sA, cA, pB, t1B, t2B, hiB, xB, sB, cB;
    const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
    const u32 c0 = (u32)c, c1 = (u32)(c >> 32), d0 = (u32)d, d1 = (u32)(d >> 32);
    asm("v_mad_u64_u32 %[pA], %[sA], %[a0], %[b0], 0\n\t"
        "v_mad_u64_u32 %[pB], %[sB], %[c0], %[d0], 0\n\t"
        "v_lshrrev_b64 %[xA], 32, %[pA]\n\t"
        "v_lshrrev_b64 %[xB], 32, %[pB]\n\t"
        "v_mad_u64_u32 %[t1A], %[sA], %[a0], %[b1], %[xA]\n\t"
        "v_mad_u64_u32 %[t1B], %[sB], %[c0], %[d1], %[xB]\n\t"
        "v_mad_u64_u32 %[t2A], %[cA], %[a1], %[b0], %[t1A]\n\t"
        "v_mad_u64_u32 %[t2B], %[cB], %[c1], %[d0], %[t1B]\n\t"
        "v_lshrrev_b64 %[xA], 32, %[t2A]\n\t"
        "v_lshrrev_b64 %[xB], 32, %[t2B]\n\t"
        "v_mad_u64_u32 %[hiA], %[sA], %[a1], %[b1], %[xA]\n\t"
        "v_mad_u64_u32 %[hiB], %[sB], %[c1], %[d1], %[xB]"
        : [pA] "=&v"(pA), [xA] "=&v"(xA), [t1A] "=&v"(t1A), [t2A] "=&v"(t2A), [hiA] "=&v"(hiA), [sA] "=&s"(sA),
          [cA] "=&s"(cA), [pB] "=&v"(pB), [xB] "=&v"(xB), [t1B] "=&v"(t1B), [t2B] "=&v"(t2B), [hiB] "=&v"(hiB),
          [sB] "=&s"(sB), [cB] "=&s"(cB)
        : [a0] "v"(a0), [a1] "v"(a1), [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1), [d0] "v"(d0),
          [d1] "v"(d1));
    u32 dA0, dA1, mA, eA0, eA1, dB0, dB1, mB, eB0, eB1;
    u64 bbA, bb2A, bbB, bb2B;
    // every VALU-written mask is read >= 2 wait states later (the other product's instruction or an s_nop 0
    // in between); cA / cB were written 4+ instructions before the statement ends
    asm("s_nop 1\n\t"
        "v_subb_co_u32_e64 %[dA0], %[bbA], %[lA0], %[hhA], %[cA]\n\t"
        "v_subb_co_u32_e64 %[dB0], %[bbB], %[lB0], %[hhB], %[cB]\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %[dA1], %[bbA], %[lA1], 0, %[bbA]\n\t"
        "v_subb_co_u32_e64 %[dB1], %[bbB], %[lB1], 0, %[bbB]\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_e64 %[mA], 0, -1, %[bbA]\n\t"
        "v_cndmask_b32_e64 %[mB], 0, -1, %[bbB]\n\t"
        "v_sub_co_u32_e64 %[eA0], %[bb2A], %[dA0], %[mA]\n\t"
        "v_sub_co_u32_e64 %[eB0], %[bb2B], %[dB0], %[mB]\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %[eA1], %[bb2A], %[dA1], 0, %[bb2A]\n\t"
        "v_subb_co_u32_e64 %[eB1], %[bb2B], %[dB1], 0, %[bb2B]"
        : [dA0] "=&v"(dA0), [dA1] "=&v"(dA1), [mA] "=&v"(mA), [eA0] "=&v"(eA0), [eA1] "=&v"(eA1), [bbA] "=&s"(bbA),
          [bb2A] "=&s"(bb2A), [dB0] "=&v"(dB0), [dB1] "=&v"(dB1), [mB] "=&v"(mB), [eB0] "=&v"(eB0), [eB1] "=&v"(eB1),
          [bbB] "=&s"(bbB), [bb2B] "=&s"(bb2B)
        : [lA0] "v"((u32)pA), [lA1] "v"((u32)t2A), [hhA] "v"((u32)(hiA >> 32)), [cA] "s"(cA), [lB0] "v"((u32)pB),
          [lB1] "v"((u32)t2B), [hhB] "v"((u32)(hiB >> 32)), [cB] "s"(cB));
    a = gl_fold(((u64)eA1 << 32) | eA0, (u32)hiA);
    c = gl_fold(((u64)eB1 << 32) | eB0, (u32)hiB);
#else
    a = gl_mul(a, b);
    c = gl_mul(c, d);
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
// a^(p - 2) = 1 / a (0 for a = 0) by an addition chain over x_k = a^(2^k - 1), x_(m+n) = x_m^(2^n) x_n:
// p - 2 = (2^32 - 2) 2^32 + (2^32 - 1), so 63 squarings and 9 multiplies instead of square-and-multiply's
// 63 + 62 (the device runs one in each proof's DEEP transcript step)
__host__ __device__ inline u64 gl_sqn(u64 x, int k) {
    for (int i = 0; i < k; i++) x = gl_mul(x, x);
    return x;
}
__host__ __device__ inline u64 gl_inv(u64 a) {
    const u64 x2 = gl_mul(gl_sqn(a, 1), a), x3 = gl_mul(gl_sqn(x2, 1), a), x6 = gl_mul(gl_sqn(x3, 3), x3);
    const u64 x12 = gl_mul(gl_sqn(x6, 6), x6), x24 = gl_mul(gl_sqn(x12, 12), x12), x30 = gl_mul(gl_sqn(x24, 6), x6);
    const u64 x31s = gl_sqn(gl_mul(gl_sqn(x30, 1), a), 1);  // a^(2^32 - 2)
    return gl_mul(gl_sqn(x31s, 32), gl_mul(x31s, a));
}
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
// (the coordinate products in pairs through gl_mul2)
__host__ __device__ __forceinline__ E2 e2_mulb(E2 x, u64 s) {
    gl_mul2(x.a, s, x.b, s);
    return x;
}
__host__ __device__ __forceinline__ E2 e2_mul(E2 x, E2 y) {
    u64 a0b0 = x.a, a1b1 = x.b;
    gl_mul2(a0b0, y.a, a1b1, y.b);
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
__host__ __device__ __forceinline__ FE<2> fe_mulb(FE<2> x, u64 s) {
    gl_mul2(x.a, s, x.b, s);
    return x;
}
__host__ __device__ __forceinline__ FE<2> fe_mul(FE<2> x, FE<2> y) {
    E2 r = e2_mul(E2{x.a, x.b}, E2{y.a, y.b});
    return FE<2>{r.a, r.b};
}

}  // namespace xfg
