// Goldilocks shift multiplies, weak add/sub and the in-register radix-2^k DFT (gfx950): shared by
// the NTT passes (ntt.hip) and the FRI fold (kernels.hip, whose size-8 inverse DFT has only
// 8th-root twiddles = powers of two).
#pragma once
#include <type_traits>
#include <utility>
#include "gl.hpp"

namespace xfg {

// ---------------------------------------------------------------- shift-based multiplies
// compile-time loops (C++17): f(std::integral_constant<int, I>) for I = 0 .. N-1, so shift amounts
// and twiddle exponents are constants at the AST level (the asm "i" operands below need that)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}
// 64-bit shifts as one v_lshlrev_b64 / v_lshrrev_b64 (the compiler splits a 64-bit shift into
// v_alignbit_b32 + a 32-bit shift: two issue slots at the same rate as the one 64-bit op)
template <int S>
__device__ __forceinline__ u64 shl64(u64 x) {
    u64 r;
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
    return r;
}
template <int S>
__device__ __forceinline__ u64 shr64(u64 x) {
    u64 r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
    return r;
}
// 32-bit shift in the e64 encoding (see add_w)
template <int S>
__device__ __forceinline__ u32 shr32(u32 x) {
    u32 r;
    asm("v_lshrrev_b32_e64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
    return r;
}
// x * 2^S mod p for 0 <= S < 96 (2^96 == -1 is handled by the caller). Canonical result for any
// u64 x when S > 0; S == 0 returns x as is.
template <int S>
__device__ __forceinline__ u64 mul_pow2(u64 x) {
    if constexpr (S == 0) {
        return x;
    } else if constexpr (S <= 32) {
        // x 2^S = lo + h 2^64 with h = x >> (64 - S) < 2^32 -> lo + h EPS
        return gl_fold(shl64<S>(x), shr32<32 - S>((u32)(x >> 32)));
    } else if constexpr (S < 64) {
        // h = x >> (64 - S) = hh 2^32 + hl -> lo + hl EPS - hh
        const u64 h = shr64<64 - S>(x);
        return gl_fold(gl_sub_u32(shl64<S>(x), (u32)(h >> 32)), (u32)h);
    } else {
        // x * 2^(S-64) = v + y * 2^32 with v < 2^32, y = x >> (96 - S) < 2^63; times 2^64 == v * EPS - y,
        // and v EPS < p, y < 2^63 keep the single borrow fold canonical
        const u32 v = (u32)x << (S - 64);
        return gl_sub_weak((u64)v * EPS, shr64<96 - S>(x));
    }
}
// exponent of two of w_{2^k} (Winterfell's roots: get_root_of_unity(k))
__host__ __device__ constexpr int root_exp2(int k) {
    return k == 1 ? 96 : k == 2 ? 48 : k == 3 ? 120 : k == 4 ? 156 : k == 5 ? 78 : k == 6 ? 39 : 0;
}
__host__ __device__ constexpr int brev_c(int x, int bits) {
    int r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

// Weakly reduced values: any u64 congruent mod p. The butterflies keep their outputs weak and
// reduce only the subtrahend / addend t (which must be < p for these forms): u + t carries at most
// once past 2^64 when t < p, and u - t borrows into a value >= EPS when t < p.
// u + t as s = u + t plus (carry) EPS. The carry out of bit 63 is bit 31 of
// (a_hi & b_hi) | ((a_hi | b_hi) & ~s_hi): one v_bitop3_b32 (truth table 0xd4 over src0, src1,
// src2 = a_hi, b_hi, s_hi) and one shift in its e64 encoding (70 T lane-ops/s against 48 for the
// VOP2 form, profiles/r05/valu_ubench.txt), then one v_mad_u64_u32 adds
// carry * EPS -- 2 half-rate + 2 full-rate instructions and no VALU -> SGPR -> VALU mask hand-off
// (the compare / cndmask form was 4 half-rate instructions plus an s_nop). No second carry: with
// t < p, s = u + t - 2^64 <= p - 2 and s + EPS < 2^64.
__device__ __forceinline__ u64 add_w(u64 a, u64 b) {  // b < p
    u64 s;
    u32 c;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(s) : "v"(a), "v"(b));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xd4\n\t"
        "v_lshrrev_b32_e64 %0, 31, %0"
        : "=&v"(c)
        : "v"((u32)(a >> 32)), "v"((u32)(b >> 32)), "v"((u32)(s >> 32)));
    return s + (u64)c * EPS;
}
__device__ __forceinline__ u64 sub_w(u64 a, u64 b) { return gl_sub_weak(a, b); }  // b < p
__device__ __forceinline__ u64 canon(u64 x) { return gl_canon(x); }

// in-register DFT of size 2^LOGR (<= 32): v[q] <- sum_r v[r] w_R^(+-rq), natural order in/out.
// In: v[r] < p for every r whose bit-reversed position is odd (the level-0 subtrahends: every
// r >= R/2), the rest may be weak. Out: weak, or canonical with CANON_OUT (the last level then
// canonicalises its minuend once and uses the canonical add / subtract: 13 VALU per butterfly
// instead of 9 plus two canonicalisations of the outputs). The shift multiplies return canonical
// values, so only the w = 1 subtrahends of levels >= 1 are reduced explicitly.
template <int LOGR, bool INV, bool CANON_OUT = false>
__device__ __forceinline__ void dft_reg(u64* v) {
    constexpr int R = 1 << LOGR;
    u64 a[R];
#pragma unroll
    for (int i = 0; i < R; i++) a[i] = v[brev_c(i, LOGR)];
    static_for<LOGR>([&](auto sc) {
        constexpr int s = decltype(sc)::value, h = 1 << s;
        static_for<R / 2>([&](auto bc) {
            constexpr int b = decltype(bc)::value;
            constexpr int pos = b & (h - 1), i0 = ((b >> s) << (s + 1)) + pos;
            constexpr int e0 = (root_exp2(s + 1) * pos) % 192;
            constexpr int e = (INV && e0) ? 192 - e0 : e0;
            // w = 2^e = -2^(e - 96) for e >= 96: the sign swaps the butterfly's add and sub
            const u64 x = a[i0 + h];
            u64 t;
            if constexpr (e % 96 != 0) t = mul_pow2<e % 96>(x);
            else if constexpr (s == 0) t = x;
            else t = canon(x);
            if constexpr (CANON_OUT && s == LOGR - 1) {
                const u64 u = canon(a[i0]);  // gl_sub_weak of canonical operands is canonical
                if constexpr (e >= 96) {
                    a[i0] = gl_sub_weak(u, t);
                    a[i0 + h] = gl_add_dev(u, t);
                } else {
                    a[i0] = gl_add_dev(u, t);
                    a[i0 + h] = gl_sub_weak(u, t);
                }
            } else {
                const u64 u = a[i0];
                if constexpr (e >= 96) {
                    a[i0] = sub_w(u, t);
                    a[i0 + h] = add_w(u, t);
                } else {
                    a[i0] = add_w(u, t);
                    a[i0 + h] = sub_w(u, t);
                }
            }
        });
    });
#pragma unroll
    for (int i = 0; i < R; i++) v[i] = a[i];
}

}  // namespace xfg
