// Host-side protocol pieces shared by the prover (prover.hip) and the verifier (verifier.cpp):
// proof options, Context elements, the Fiat-Shamir coin, batch Merkle opening plans.
// Winterfell 0.8.3 as restated in DESIGN.md "Proof format and transcript".
#pragma once
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "../../include/xfg_stark.h"
#include "gl.hpp"
#include "host_crypto.hpp"

namespace xfg {

static inline unsigned ilog2(u64 x) {
    unsigned r = 0;
    while ((1ULL << r) < x) r++;
    return r;
}
static inline bool is_pow2(u64 x) { return x && !(x & (x - 1)); }

// ------------------------------------------------------------------ options / context elements
struct Opts {
    u64 q, beta, grind, ext, fold, remdeg;
};
static inline Opts to_opts(const xfg_options* o) {
    return Opts{o->num_queries, o->blowup_factor, o->grinding_factor, o->field_extension, o->fri_folding_factor,
                o->fri_remainder_max_degree};
}
// ProofOptions::new validation (winter-air 0.8) + what this GPU path implements
static inline const char* check_options(u64 n, const Opts& o) {
    if (!is_pow2(n) || n < 8) return "trace length must be a power of two and at least 8";
    if (n > (1ULL << 21)) return "trace length above 2^21 is not supported";
    if (!is_pow2(o.beta) || o.beta < 2 || o.beta > 16) return "blowup factor must be a power of two in [2, 16]";
    if (o.q < 1 || o.q > 255) return "number of queries must be in [1, 255]";
    if (o.grind > 32) return "grinding factor cannot be greater than 32";
    if (o.ext != 1 && o.ext != 2) return "field extension must be None (1) or Quadratic (2)";
    if (o.fold != 8) return "only FRI folding factor 8 is supported by this prover";
    if (o.remdeg > 255 || !is_pow2(o.remdeg + 1)) return "FRI remainder max degree must be one less than a power of two";
    if (o.q >= n * o.beta) return "number of queries must be smaller than the LDE domain size";
    return nullptr;
}
static inline unsigned num_fri_layers(u64 N, const Opts& o) {
    u64 maxrem = (o.remdeg + 1) * o.beta;
    unsigned k = 0;
    while (N > maxrem) {
        N /= o.fold;
        k++;
    }
    return k;
}
// Context::to_elements (TraceInfo, modulus bytes, options) -- DESIGN.md "Transcript"
static inline void context_elements(u64 n, const Opts& o, u64* e) {
    e[0] = 7ULL << 8;
    e[1] = n;
    e[2] = 1;
    e[3] = 0xFFFFFFFFULL;
    e[4] = (o.ext << 16) | (o.fold << 8) | o.remdeg;
    e[5] = o.grind;
    e[6] = o.beta;
    e[7] = o.q;
}

// ------------------------------------------------------------------ DefaultRandomCoin<Blake3_256>
struct Coin {
    Digest seed;
    u64 counter = 0;
    void init(const u64* e, size_t cnt) {
        seed = hash_elements(e, cnt);
        counter = 0;
    }
    void reseed(const Digest& d) {
        seed = b3_merge(seed, d);
        counter = 0;
    }
    void reseed_int(u64 v) {
        seed = merge_with_int(seed, v);
        counter = 0;
    }
    Digest next() { return merge_with_int(seed, ++counter); }
    bool draw(u64& out) {
        for (int i = 0; i < 1000; i++) {
            Digest v = next();
            u64 x = (u64)v.w[0] | ((u64)v.w[1] << 32);
            if (x < P) {
                out = x;
                return true;
            }
        }
        return false;
    }
    // draw::<E>() for extension degree d: the first 8 d digest bytes as d LE elements, retried
    // while any of them is >= p (QuadExtension::from_random_bytes); out[d]
    bool draw_e(u64* out, int d) {
        if (d == 1) return draw(out[0]);
        for (int i = 0; i < 1000; i++) {
            Digest v = next();
            const u64 x = (u64)v.w[0] | ((u64)v.w[1] << 32), y = (u64)v.w[2] | ((u64)v.w[3] << 32);
            if (x < P && y < P) {
                out[0] = x;
                out[1] = y;
                return true;
            }
        }
        return false;
    }
};
static inline unsigned tz64(u64 x) { return x ? (unsigned)__builtin_ctzll(x) : 64; }


// ------------------------------------------------------------------ batch Merkle openings
// MerkleTree::prove_batch (winter-crypto 0.8.3) restated as heap-index lists: node vector i holds
// the missing sibling leaf of normalised pair i, then the siblings met by the i-th entry of each
// upper level's index list. Digests are gathered from HBM afterwards in this order.
struct BatchOpening {
    // node vector i = node[i * stride .. i * stride + len[i]) (heap indices, leaf i -> L + i)
    u64 stride = 0;
    std::vector<u64> node;
    std::vector<uint8_t> len;
    size_t size() const { return len.size(); }
    const u64* row(size_t i) const { return node.data() + i * stride; }
    template <class F>
    void each(F f) const {
        for (size_t i = 0; i < len.size(); i++)
            for (unsigned k = 0; k < len[i]; k++) f(node[i * stride + k]);
    }
};
static inline void plan_batch_opening(const std::vector<u64>& idx, u64 L, BatchOpening& op) {
    unsigned depth = ilog2(L);
    u64 cur[256], sorted[256];  // idx.size() <= num_queries <= 255
    size_t cnt = idx.size();
    std::copy(idx.begin(), idx.end(), sorted);
    std::sort(sorted, sorted + cnt);
    size_t nn = 0;
    for (size_t i = 0; i < cnt; i++) {
        u64 v = sorted[i] & ~1ULL;
        if (nn == 0 || cur[nn - 1] != v) cur[nn++] = v;
    }
    op.stride = depth + 1;
    op.len.assign(nn, 0);
    op.node.resize(nn * op.stride);
    auto push = [&](size_t i, u64 h) { op.node[i * op.stride + op.len[i]++] = h; };
    for (size_t i = 0; i < nn; i++) {
        for (u64 leaf = cur[i]; leaf < cur[i] + 2; leaf++)
            if (!std::binary_search(sorted, sorted + cnt, leaf)) push(i, L + leaf);
        cur[i] = (cur[i] + L) >> 1;
    }
    for (unsigned lvl = 1; lvl < depth; lvl++) {
        size_t m = 0;
        for (size_t i = 0; i < nn; i++) {
            u64 sib = cur[i] ^ 1;
            if (i + 1 < nn && cur[i + 1] == sib) i++;
            else push(i, sib);
            cur[m++] = sib >> 1;  // m <= i: in-place compaction is safe
        }
        nn = m;
    }
}
static inline std::vector<u64> fold_positions(const std::vector<u64>& in, u64 target) {
    std::vector<u64> out;
    out.reserve(in.size());
    for (u64 p : in) {
        u64 q = p & (target - 1);  // target is a power of two
        if (std::find(out.begin(), out.end(), q) == out.end()) out.push_back(q);
    }
    return out;
}


}  // namespace xfg
