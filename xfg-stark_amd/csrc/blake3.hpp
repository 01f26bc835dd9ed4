// BLAKE3 compression for the Merkle commitments and Fiat-Shamir transcript of the burn-proof
// STARK (winter-crypto `Blake3_256`, reference src/burn_mint_air.rs:483-485).
// Everything on the hot path is a single 64-byte-or-shorter block: leaf = one trace row
// (7 elements = 56 B), FRI leaf = 8 elements (64 B), Merkle node = two digests (64 B),
// coin step = digest||u64 (40 B). Digests are 8 little-endian u32 words, so field elements map
// to message words directly (lo, hi) -- no byte shuffling on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xfg {

struct Digest {
    uint32_t w[8];
};

#define XFG_B3_IV0 0x6A09E667u
#define XFG_B3_IV1 0xBB67AE85u
#define XFG_B3_IV2 0x3C6EF372u
#define XFG_B3_IV3 0xA54FF53Au
#define XFG_B3_IV4 0x510E527Fu
#define XFG_B3_IV5 0x9B05688Cu
#define XFG_B3_IV6 0x1F83D9ABu
#define XFG_B3_IV7 0x5BE0CD19u

enum : uint32_t { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };

__host__ __device__ __forceinline__ uint32_t b3_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// xor / add of two variables in their VOP3 (e64) encodings: v_xor_b32_e64 issues at 65 T lane-ops/s
// against 47 for the VOP2 form (profiles/r05/valu_ubench.txt), and BLAKE3 with both its xors and its
// two-input adds in the e64 encoding ran the leaf kernels 6-10 % faster and the bench 5 % faster
// (profiles/r05/b3_vop3_ab.txt). Operands the compiler knows are constants keep the plain C form
// so that it still folds them (the first round's IV words, zero message words).
__host__ __device__ __forceinline__ uint32_t b3_xor(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_constant_p(a) || __builtin_constant_p(b)) return a ^ b;
    uint32_t r;
    asm("v_xor_b32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return a ^ b;
#endif
}
__host__ __device__ __forceinline__ uint32_t b3_add(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_constant_p(a) || __builtin_constant_p(b)) return a + b;
    uint32_t r;
    asm("v_add_u32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return a + b;
#endif
}

// a + b + x: v_add3_u32, or the e64 add when the message word is a known zero (padding words)
__host__ __device__ __forceinline__ uint32_t b3_add3(uint32_t a, uint32_t b, uint32_t x) {
    if (__builtin_constant_p(x) && x == 0) return b3_add(a, b);
    return a + b + x;
}

#define XFG_B3_G(a, b, c, d, x, y)                    \
    do {                                              \
        s[a] = b3_add3(s[a], s[b], (x));              \
        s[d] = b3_rotr(b3_xor(s[d], s[a]), 16);       \
        s[c] = b3_add(s[c], s[d]);                    \
        s[b] = b3_rotr(b3_xor(s[b], s[c]), 12);       \
        s[a] = b3_add3(s[a], s[b], (y));              \
        s[d] = b3_rotr(b3_xor(s[d], s[a]), 8);        \
        s[c] = b3_add(s[c], s[d]);                    \
        s[b] = b3_rotr(b3_xor(s[b], s[c]), 7);        \
    } while (0)

// one round with message words already permuted into m[] (compiler-scheduled): column half, then
// diagonal half
#define XFG_B3_COL_C(m)                                   \
    do {                                                  \
        XFG_B3_G(0, 4, 8, 12, m[0], m[1]);                \
        XFG_B3_G(1, 5, 9, 13, m[2], m[3]);                \
        XFG_B3_G(2, 6, 10, 14, m[4], m[5]);               \
        XFG_B3_G(3, 7, 11, 15, m[6], m[7]);               \
    } while (0)
#define XFG_B3_DIAG_C(m)                                  \
    do {                                                  \
        XFG_B3_G(0, 5, 10, 15, m[8], m[9]);               \
        XFG_B3_G(1, 6, 11, 12, m[10], m[11]);             \
        XFG_B3_G(2, 7, 8, 13, m[12], m[13]);              \
        XFG_B3_G(3, 4, 9, 14, m[14], m[15]);              \
    } while (0)
#define XFG_B3_ROUND_C(m) \
    do {                  \
        XFG_B3_COL_C(m);  \
        XFG_B3_DIAG_C(m); \
    } while (0)

// BLAKE3 message permutation applied in registers between rounds (compile-time indices)
#define XFG_B3_PERMUTE(m)                                                                   \
    do {                                                                                    \
        uint32_t t0 = m[0], t1 = m[1], t2 = m[2], t3 = m[3], t4 = m[4], t5 = m[5], t6 = m[6], \
                 t7 = m[7], t8 = m[8], t9 = m[9], t10 = m[10], t11 = m[11], t12 = m[12],      \
                 t13 = m[13], t14 = m[14], t15 = m[15];                                     \
        m[0] = t2; m[1] = t6; m[2] = t3; m[3] = t10; m[4] = t7; m[5] = t0; m[6] = t4;        \
        m[7] = t13; m[8] = t1; m[9] = t11; m[10] = t12; m[11] = t5; m[12] = t9; m[13] = t14; \
        m[14] = t15; m[15] = t8;                                                            \
    } while (0)

// the same permutation as a constexpr map on zero masks: round r + 1 reads m'[i] = m[P[i]]
__host__ __device__ constexpr unsigned b3_perm_mask(unsigned z) {
    constexpr int P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
    unsigned r = 0;
    for (int i = 0; i < 16; i++) r |= ((z >> P[i]) & 1u) << i;
    return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// The device rounds 2-7 issue in a fixed order: each half-round (four independent G functions, 48
// VALU) is one asm block generated by scripts/b3_sched_gen.py -- fast and slow instructions of
// different G's alternating, an s_nop after each fast one. gfx950 issues its two-source e64 xor / add
// about 1.7x faster than add3 / alignbit, and how close a mix of the two gets to its harmonic rate
// depends on the order: the compiler's order of the same 680 instructions per compression issues at
// 35-37 T lane-instructions/s, fixed orders at 40-42 without s_nops and 42-45 with them
// (profiles/r05/b3_sched.txt). Message words known to be zero (the padding of short element hashes,
// tracked through the permutation as the mask Z) select a block whose add3 for that word is a fast
// two-source add. No operand can alias another: every state word a block reads is an output of the
// C column half or of the previous block, and the message words are read-only.
#include "b3_sched.inc"
#define XFG_B3_DIAG_Z(m, Z)                                                                          \
    b3_half<((Z) >> 8) & 0xFFu>(s[0], s[5], s[10], s[15], s[1], s[6], s[11], s[12], s[2], s[7], s[8], s[13], \
                                s[3], s[4], s[9], s[14], m[8], m[9], m[10], m[11], m[12], m[13], m[14], m[15])
#define XFG_B3_ROUND_Z(m, Z)                                                                         \
    do {                                                                                             \
        b3_half<(Z) & 0xFFu>(s[0], s[4], s[8], s[12], s[1], s[5], s[9], s[13], s[2], s[6], s[10], s[14],  \
                             s[3], s[7], s[11], s[15], m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);   \
        XFG_B3_DIAG_Z(m, Z);                                                                         \
    } while (0)
#else  // host: the compiler's order
#define XFG_B3_DIAG_Z(m, Z) XFG_B3_DIAG_C(m)
#define XFG_B3_ROUND_Z(m, Z) XFG_B3_ROUND_C(m)
#endif

// compression returning the first 8 output words (chaining value / digest); ZM: message words known
// to be zero (bit i = m[i]), a compile-time hint for the device rounds (any value is correct for 0)
template <unsigned ZM = 0>
__host__ __device__ __forceinline__ void b3_compress(const uint32_t cv[8], uint32_t m[16], uint32_t block_len,
                                                     uint64_t counter, uint32_t flags, uint32_t out[8]) {
    uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3,
                      (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags};
    [[maybe_unused]] constexpr unsigned Z2 = b3_perm_mask(ZM), Z3 = b3_perm_mask(Z2), Z4 = b3_perm_mask(Z3),
                       Z5 = b3_perm_mask(Z4), Z6 = b3_perm_mask(Z5), Z7 = b3_perm_mask(Z6);
    // round 1: the column half in C (the IV / counter / flag words of the state fold into it); the
    // diagonal half as a block too, unless a column G had no message (both words zero): its outputs
    // are then compile-time constants the C diagonal half folds (short element hashes)
    constexpr bool col_const = (ZM & 0x03u) == 0x03u || (ZM & 0x0Cu) == 0x0Cu || (ZM & 0x30u) == 0x30u ||
                               (ZM & 0xC0u) == 0xC0u;
    XFG_B3_COL_C(m);
    if constexpr (col_const)
        XFG_B3_DIAG_C(m);
    else
        XFG_B3_DIAG_Z(m, ZM);
    XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z2); XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z3); XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z4); XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z5); XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z6); XFG_B3_PERMUTE(m);
    XFG_B3_ROUND_Z(m, Z7);
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = b3_xor(s[i], s[i + 8]);
}

// BLAKE3 of a single block of `len` (<= 64) bytes given as 16 LE words (zero padded)
template <unsigned ZM = 0>
__host__ __device__ __forceinline__ Digest b3_hash_block(uint32_t m[16], uint32_t len) {
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3,
                            XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    Digest d;
    b3_compress<ZM>(iv, m, len, 0, B3_CHUNK_START | B3_CHUNK_END | B3_ROOT, d.w);
    return d;
}
// Blake3_256::merge([a, b]) = BLAKE3(a || b)
__host__ __device__ __forceinline__ Digest b3_merge(const Digest& a, const Digest& b) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { m[i] = a.w[i]; m[8 + i] = b.w[i]; }
    return b3_hash_block(m, 64);
}
// Blake3_256::hash_elements for up to 16 field elements (one or two blocks of one chunk)
template <int K>
__host__ __device__ __forceinline__ Digest b3_hash_elems(const uint64_t* e) {
    static_assert(K >= 1 && K <= 16, "one- or two-block element hash");
    uint32_t m[16];
    constexpr int K0 = K <= 8 ? K : 8;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t v = i < K0 ? e[i] : 0;
        m[2 * i] = (uint32_t)v;
        m[2 * i + 1] = (uint32_t)(v >> 32);
    }
    if constexpr (K <= 8) {
        return b3_hash_block<0xFFFFu & ~((1u << (2 * K)) - 1u)>(m, 8 * K);  // words 2K.. are zero
    } else {
        const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3,
                                XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
        uint32_t cv[8];
        b3_compress(iv, m, 64, 0, B3_CHUNK_START, cv);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint64_t v = 8 + i < K ? e[8 + i] : 0;
            m[2 * i] = (uint32_t)v;
            m[2 * i + 1] = (uint32_t)(v >> 32);
        }
        Digest d;
        b3_compress<0xFFFFu & ~((1u << (2 * (K - 8))) - 1u)>(cv, m, 8 * (K - 8), 0, B3_CHUNK_END | B3_ROOT, d.w);
        return d;
    }
}

}  // namespace xfg
