// Host-side hashing for the transcript and AIR constants (product code; the parity oracle under
// oracle/ is a separate, independent C restatement).
//  - BLAKE3 (any length; transcript inputs are one chunk except FRI remainders > 128 elements):
//    Fiat-Shamir seed (Context || public inputs, 160 B),
//    OOD frame hash (112 B), FRI remainder commitment, coin draws.
//  - Keccak-256 (sha3::Keccak256): AIR constants, reference src/burn_mint_air.rs:124-202 and
//    src/burn_mint_prover.rs:211-221 -- computed once per proof instead of once per
//    constraint-evaluation row as the reference does (:264, :376); values are identical.
#pragma once
#include <stdint.h>
#include <string.h>
#include <array>
#include <vector>
#include "blake3.hpp"

namespace xfg {

inline void le_words(const uint8_t* b, size_t len, uint32_t m[16]) {
    for (int i = 0; i < 16; i++) m[i] = 0;
    for (size_t i = 0; i < len; i++) m[i / 4] |= (uint32_t)b[i] << (8 * (i % 4));
}
// BLAKE3 (hash mode, any length): 1024-byte chunks chained block by block; chunk chaining values
// merged in the left-balanced binary tree of the BLAKE3 spec (PARENT nodes), ROOT on the last
// compression. One-chunk inputs (every transcript hash except long FRI remainders) take the
// first branch only.
struct B3Output {  // a compression whose flags are not final yet (ROOT is added at the very end)
    uint32_t cv[8], m[16], len, flags;
    uint64_t counter;
    void chaining(uint32_t out[8]) const {
        uint32_t mm[16];
        memcpy(mm, m, sizeof mm);
        b3_compress(cv, mm, len, counter, flags, out);
    }
    Digest root() const {
        uint32_t mm[16];
        memcpy(mm, m, sizeof mm);
        Digest d;
        b3_compress(cv, mm, len, counter, flags | B3_ROOT, d.w);
        return d;
    }
};
inline B3Output b3_chunk(const uint8_t* in, size_t len, uint64_t counter) {
    B3Output o;
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    memcpy(o.cv, iv, sizeof iv);
    const size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < nblocks; b++) {
        const size_t off = b * 64, bl = len == 0 ? 0 : (len - off < 64 ? len - off : 64);
        le_words(in + off, bl, o.m);
        o.len = (uint32_t)bl;
        o.counter = counter;
        o.flags = (b == 0 ? B3_CHUNK_START : 0) | (b == nblocks - 1 ? B3_CHUNK_END : 0);
        if (b + 1 < nblocks) {
            uint32_t out[8];
            o.chaining(out);
            memcpy(o.cv, out, sizeof out);
        }
    }
    return o;
}
inline B3Output b3_parent(const uint32_t l[8], const uint32_t r[8]) {
    B3Output o;
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    memcpy(o.cv, iv, sizeof iv);
    memcpy(o.m, l, 32);
    memcpy(o.m + 8, r, 32);
    o.len = 64;
    o.counter = 0;
    o.flags = B3_PARENT;
    return o;
}
inline Digest blake3_bytes(const uint8_t* in, size_t len) {
    const size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
    std::vector<std::array<uint32_t, 8>> stack;
    for (size_t c = 0; c + 1 < nchunks; c++) {
        std::array<uint32_t, 8> cv;
        b3_chunk(in + c * 1024, 1024, c).chaining(cv.data());
        for (uint64_t total = c + 1; (total & 1) == 0; total >>= 1) {  // add_chunk_chaining_value
            std::array<uint32_t, 8> merged;
            b3_parent(stack.back().data(), cv.data()).chaining(merged.data());
            stack.pop_back();
            cv = merged;
        }
        stack.push_back(cv);
    }
    const size_t last = (nchunks - 1) * 1024;
    B3Output out = b3_chunk(in + last, len - last, nchunks - 1);
    while (!stack.empty()) {
        uint32_t cv[8];
        out.chaining(cv);
        out = b3_parent(stack.back().data(), cv);
        stack.pop_back();
    }
    return out.root();
}
inline void digest_bytes(const Digest& d, uint8_t out[32]) {
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(d.w[i] >> (8 * j));
}
inline Digest hash_elements(const uint64_t* e, size_t cnt) {
    std::vector<uint8_t> b(cnt * 8);
    for (size_t i = 0; i < cnt; i++)
        for (int j = 0; j < 8; j++) b[8 * i + j] = (uint8_t)(e[i] >> (8 * j));
    return blake3_bytes(b.data(), b.size());
}
inline Digest merge_with_int(const Digest& seed, uint64_t v) {
    uint32_t m[16];
    for (int i = 0; i < 8; i++) m[i] = seed.w[i];
    m[8] = (uint32_t)v;
    m[9] = (uint32_t)(v >> 32);
    for (int i = 10; i < 16; i++) m[i] = 0;
    return b3_hash_block(m, 40);
}

// ---------------------------------------------------------------- Keccak-256
namespace keccak_detail {
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
// rotation offsets and pi-lane order of the lane-walk formulation
static const int ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
static const int PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
inline uint64_t rol(uint64_t x, int s) { return (x << s) | (x >> (64 - s)); }
inline void permute(uint64_t st[25]) {
    for (int r = 0; r < 24; r++) {
        uint64_t bc[5];
        for (int i = 0; i < 5; i++) bc[i] = st[i] ^ st[i + 5] ^ st[i + 10] ^ st[i + 15] ^ st[i + 20];
        for (int i = 0; i < 5; i++) {
            uint64_t t = bc[(i + 4) % 5] ^ rol(bc[(i + 1) % 5], 1);
            for (int j = 0; j < 25; j += 5) st[j + i] ^= t;
        }
        uint64_t t = st[1];
        for (int i = 0; i < 24; i++) {
            int j = PILN[i];
            uint64_t tmp = st[j];
            st[j] = rol(t, ROTC[i]);
            t = tmp;
        }
        for (int j = 0; j < 25; j += 5) {
            uint64_t b[5];
            for (int i = 0; i < 5; i++) b[i] = st[j + i];
            for (int i = 0; i < 5; i++) st[j + i] ^= (~b[(i + 1) % 5]) & b[(i + 2) % 5];
        }
        st[0] ^= RC[r];
    }
}
}  // namespace keccak_detail

inline void keccak256(const uint8_t* in, size_t len, uint8_t out[32]) {
    const size_t rate = 136;
    uint64_t st[25] = {0};
    std::vector<uint8_t> msg(in, in + len);
    size_t padded = (len / rate + 1) * rate;
    msg.resize(padded, 0);
    msg[len] ^= 0x01;
    msg[padded - 1] ^= 0x80;
    for (size_t off = 0; off < padded; off += rate) {
        for (size_t i = 0; i < rate / 8; i++) {
            uint64_t w = 0;
            for (int j = 0; j < 8; j++) w |= (uint64_t)msg[off + 8 * i + j] << (8 * j);
            st[i] ^= w;
        }
        keccak_detail::permute(st);
    }
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
}

}  // namespace xfg
