/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 * This directory is the CPU parity oracle for the XFG burn-proof STARK path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (xfg-stark_amd/, include/) never links or calls it.
 *
 * orc_prims.h -- Goldilocks field, BLAKE3, Keccak-256 (plain C restatements).
 *
 * Field: Winterfell `math::fields::f64::BaseElement` (reference src/burn_mint_air.rs:17),
 *   p = 2^64 - 2^32 + 1, generator 7, two-adicity 32,
 *   2^32-th root of unity 1753635133440165772 (= 7^((p-1)/2^32)); canonical LE u64 encoding.
 * BLAKE3: winter-crypto `Blake3_256` over blake3 1.8.2 (reference src/burn_mint_air.rs:483);
 *   pinned by the published BLAKE3 test vectors (tests/golden/kat_blake3.json).
 * Keccak-256: sha3 0.10 `Keccak256` (reference src/burn_mint_air.rs:14,124-202);
 *   pinned by the reference's own KAT src/lib.rs:135-161 and the Keccak spec vectors.
 */
#ifndef ORC_PRIMS_H
#define ORC_PRIMS_H
#include <stdint.h>
#include <stddef.h>

#define ORC_P 0xFFFFFFFF00000001ULL
#define ORC_GEN 7ULL
#define ORC_TWO_ADIC_ROOT 1753635133440165772ULL

typedef unsigned __int128 orc_u128;

static inline uint64_t orc_add(uint64_t a, uint64_t b) {
    orc_u128 s = (orc_u128)a + b;
    if (s >= ORC_P) s -= ORC_P;
    return (uint64_t)s;
}
static inline uint64_t orc_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (ORC_P - b); }
static inline uint64_t orc_neg(uint64_t a) { return a ? ORC_P - a : 0; }
/* reduction of a 128-bit product using 2^64 = 2^32 - 1 and 2^96 = -1 (mod p) */
static inline uint64_t orc_reduce128(orc_u128 x) {
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    uint64_t hi_hi = hi >> 32, hi_lo = hi & 0xFFFFFFFFULL;
    uint64_t t0 = lo - hi_hi;
    if (lo < hi_hi) t0 -= 0xFFFFFFFFULL; /* borrow: -2^64 == -(2^32-1) */
    uint64_t t1 = hi_lo * 0xFFFFFFFFULL;
    uint64_t t2 = t0 + t1;
    if (t2 < t1) t2 += 0xFFFFFFFFULL; /* carry: +2^64 == +(2^32-1) */
    if (t2 >= ORC_P) t2 -= ORC_P;
    return t2;
}
static inline uint64_t orc_mul(uint64_t a, uint64_t b) { return orc_reduce128((orc_u128)a * b); }
static inline uint64_t orc_pow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r = orc_mul(r, b); b = orc_mul(b, b); e >>= 1; }
    return r;
}
static inline uint64_t orc_inv(uint64_t a) { return orc_pow(a, ORC_P - 2); }
/* primitive 2^k-th root of unity, winter-math `get_root_of_unity(k)` */
static inline uint64_t orc_root(unsigned k) { return orc_pow(ORC_TWO_ADIC_ROOT, 1ULL << (32 - k)); }

/* BLAKE3 (default hash mode, 32-byte output) */
void orc_blake3(const uint8_t* in, size_t len, uint8_t out[32]);
/* Keccak-256 (original Keccak padding 0x01, as sha3::Keccak256) */
void orc_keccak256(const uint8_t* in, size_t len, uint8_t out[32]);
/* generic sponge used by tests to check the permutation against hashlib.sha3_256 (pad 0x06) */
void orc_keccak_sponge(const uint8_t* in, size_t len, uint8_t pad, uint8_t out[32]);

#endif
