/*
 * ORACLE / TEST INFRASTRUCTURE ONLY (see orc_prims.h).
 * BLAKE3 and Keccak-256 restated from their published specifications.
 *  - BLAKE3: used by winter-crypto 0.8.3 `Blake3_256` (reference src/burn_mint_air.rs:483-485),
 *    blake3 crate 1.8.2 (version pin: SURVEY.md §0.1). Full tree mode (multi-chunk) implemented.
 *  - Keccak-256: sha3 0.10 `Keccak256` as used at reference src/burn_mint_air.rs:124-202 and
 *    src/burn_mint_prover.rs:211-221.
 */
#include <string.h>
#include "orc_prims.h"

/* ------------------------------------------------------------------ BLAKE3 */
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline void b3_g(uint32_t* s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    s[a] = s[a] + s[b] + x; s[d] = rotr32(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];     s[b] = rotr32(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + y; s[d] = rotr32(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];     s[b] = rotr32(s[b] ^ s[c], 7);
}
static void b3_compress(const uint32_t cv[8], const uint8_t block[64], uint32_t block_len,
                        uint64_t counter, uint32_t flags, uint32_t out[16]) {
    uint32_t m[16], s[16], t[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) |
               ((uint32_t)block[4 * i + 2] << 16) | ((uint32_t)block[4 * i + 3] << 24);
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    for (int i = 0; i < 4; i++) s[8 + i] = B3_IV[i];
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32); s[14] = block_len; s[15] = flags;
    for (int r = 0; r < 7; r++) {
        b3_g(s, 0, 4, 8, 12, m[0], m[1]);  b3_g(s, 1, 5, 9, 13, m[2], m[3]);
        b3_g(s, 2, 6, 10, 14, m[4], m[5]); b3_g(s, 3, 7, 11, 15, m[6], m[7]);
        b3_g(s, 0, 5, 10, 15, m[8], m[9]); b3_g(s, 1, 6, 11, 12, m[10], m[11]);
        b3_g(s, 2, 7, 8, 13, m[12], m[13]); b3_g(s, 3, 4, 9, 14, m[14], m[15]);
        if (r < 6) { for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]]; memcpy(m, t, sizeof m); }
    }
    for (int i = 0; i < 8; i++) { out[i] = s[i] ^ s[i + 8]; out[i + 8] = s[i + 8] ^ cv[i]; }
}
/* chaining value of one chunk (<=1024 bytes); is_root applies ROOT to the last block */
static void b3_chunk_cv(const uint8_t* in, size_t len, uint64_t chunk_idx, int is_root, uint32_t cv_out[8]) {
    uint32_t cv[8], out[16];
    memcpy(cv, B3_IV, sizeof cv);
    size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < nblocks; b++) {
        uint8_t block[64] = {0};
        size_t off = b * 64, bl = len - off < 64 ? len - off : 64;
        if (len == 0) bl = 0;
        memcpy(block, in + off, bl);
        uint32_t flags = 0;
        if (b == 0) flags |= CHUNK_START;
        if (b == nblocks - 1) { flags |= CHUNK_END; if (is_root) flags |= ROOT; }
        b3_compress(cv, block, (uint32_t)bl, chunk_idx, flags, out);
        memcpy(cv, out, sizeof cv);
    }
    memcpy(cv_out, cv, sizeof cv);
}
static void b3_parent_cv(const uint32_t l[8], const uint32_t r[8], int is_root, uint32_t cv_out[8]) {
    uint8_t block[64];
    uint32_t out[16];
    for (int i = 0; i < 8; i++) for (int j = 0; j < 4; j++) {
        block[4 * i + j] = (uint8_t)(l[i] >> (8 * j));
        block[32 + 4 * i + j] = (uint8_t)(r[i] >> (8 * j));
    }
    b3_compress(B3_IV, block, 64, 0, PARENT | (is_root ? ROOT : 0), out);
    memcpy(cv_out, out, 32);
}
/* subtree of a power-of-two number of whole chunks (left-subtree rule of the spec) */
static void b3_subtree(const uint8_t* in, size_t len, uint64_t chunk0, int is_root, uint32_t cv[8]) {
    if (len <= 1024) { b3_chunk_cv(in, len, chunk0, is_root, cv); return; }
    size_t left = 1024; /* largest power-of-two number of chunks strictly less than total */
    while (left * 2 < len) left *= 2;
    uint32_t l[8], r[8];
    b3_subtree(in, left, chunk0, 0, l);
    b3_subtree(in + left, len - left, chunk0 + left / 1024, 0, r);
    b3_parent_cv(l, r, is_root, cv);
}
void orc_blake3(const uint8_t* in, size_t len, uint8_t out[32]) {
    uint32_t cv[8];
    b3_subtree(in, len, 0, 1, cv);
    for (int i = 0; i < 8; i++) for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(cv[i] >> (8 * j));
}

/* ------------------------------------------------------------------ Keccak */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static inline uint64_t rotl64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }
static void keccak_f(uint64_t a[25]) {
    static const int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; round++) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
        /* rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y]) */
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], rho[x + 5 * y]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++)
                a[x + 5 * y] = b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= KRC[round];
    }
}
void orc_keccak_sponge(const uint8_t* in, size_t len, uint8_t pad, uint8_t out[32]) {
    const size_t rate = 136;
    uint64_t st[25] = {0};
    uint8_t block[136];
    for (;;) {
        size_t take = len < rate ? len : rate;
        memset(block, 0, rate);
        memcpy(block, in, take);
        int last = take < rate;
        if (last) { block[take] ^= pad; block[rate - 1] ^= 0x80; }
        for (size_t i = 0; i < rate / 8; i++) {
            uint64_t w = 0;
            for (int j = 0; j < 8; j++) w |= (uint64_t)block[8 * i + j] << (8 * j);
            st[i] ^= w;
        }
        keccak_f(st);
        in += take; len -= take;
        if (last) break;
    }
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
}
void orc_keccak256(const uint8_t* in, size_t len, uint8_t out[32]) { orc_keccak_sponge(in, len, 0x01, out); }
