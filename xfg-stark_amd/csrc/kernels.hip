// HIP kernels (CDNA4 / gfx950) for the XFG burn-proof STARK hot path.
//
// Replaces, inside Winterfell 0.8.3 `Prover::prove` as bound by the reference
// (src/burn_mint_air.rs:479-531, called at src/burn_mint_prover.rs:124-126):
//   - DefaultTraceLde: column interpolation + coset LDE (four-step NTT, LDS radix-2 stages)
//   - RowMatrix::commit_to_rows / MerkleTree::new: Blake3 row hashing + binary Merkle tree
//   - DefaultConstraintEvaluator with XfgBurnMintAir::evaluate_transition (:335-378) and the
//     8 assertions (:380-395), batch-inverted divisors
//   - CompositionPoly / DeepCompositionPoly: OOD evaluation, coefficient-domain DEEP combine with
//     synthetic division expressed as a weighted suffix scan
//   - FriProver::build_layers: fold-by-8 (apply_drp) and per-layer commitments
// All arithmetic is 64-bit Goldilocks integer work: HBM/VALU bound, no MFMA.
#include "kernels.hpp"
#include "field_dft.hpp"
#include <algorithm>

namespace xfg {

#define XFG_CHECK_LAUNCH() (void)hipGetLastError()

__device__ __forceinline__ unsigned brev(unsigned x, int bits) { return __brev(x) >> (32 - bits); }

// w_{2^k}^e from the master table (forward) / its inverse
__device__ __forceinline__ u64 tw_pow(const Tables& T, int k, u64 e) {
    u64 M = 1ULL << T.LM;
    return T.tw[(e << (T.LM - k)) & (M - 1)];
}
__device__ __forceinline__ u64 tw_ipow(const Tables& T, int k, u64 e) {
    u64 M = 1ULL << T.LM;
    return T.tw[(M - ((e << (T.LM - k)) & (M - 1))) & (M - 1)];
}

// One Merkle parent BLAKE3(l || r) (one 64-byte block: CHUNK_START | CHUNK_END | ROOT, counter 0) computed
// by the four lanes of a quad: lane q holds column q of the state (s[q], s[4 + q], s[8 + q], s[12 + q]) and
// all 16 message words. The column half is lane q's G function on its own column; for the diagonal half
// rows 1-3 rotate by 1, 2, 3 lanes (DPP quad_perm, the compiler's hazard padding) so that lane q holds
// s[q], s[4 + (q+1)%4], s[8 + (q+2)%4], s[12 + (q+3)%4], and rotate back after it. Each lane picks its
// G's two message words of the round by a 4-way select. ~330 VALU per lane on the critical path instead of
// one lane's ~680: the serial top levels of a tree (one compression per level) finish about twice as
// fast, at four lanes per node. Returns (out[q], out[4 + q]).
__device__ __forceinline__ uint32_t sel4(bool b0, bool b1, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    return b1 ? (b0 ? x3 : x2) : (b0 ? x1 : x0);
}
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
constexpr int QP_ROT1 = 0x39, QP_ROT2 = 0x4E, QP_ROT3 = 0x93;  // lane q reads lane (q + k) % 4
#define XFG_B3_GQ(a, b, c, d, x, y)               \
    do {                                          \
        a = b3_add3(a, b, (x));                   \
        d = b3_rotr(b3_xor(d, a), 16);            \
        c = b3_add(c, d);                         \
        b = b3_rotr(b3_xor(b, c), 12);            \
        a = b3_add3(a, b, (y));                   \
        d = b3_rotr(b3_xor(d, a), 8);             \
        c = b3_add(c, d);                         \
        b = b3_rotr(b3_xor(b, c), 7);             \
    } while (0)
// (any chaining value, block length and flags, counter 0: b3_compress_quad; the Merkle parent: b3_merge_quad)
__device__ __forceinline__ uint2 b3_compress_quad(const uint32_t cv[8], uint32_t m[16], uint32_t len, uint32_t flags,
                                                  int q) {
    const bool q0 = q & 1, q1 = (q & 2) != 0;
    uint32_t a = sel4(q0, q1, cv[0], cv[1], cv[2], cv[3]);
    uint32_t b = sel4(q0, q1, cv[4], cv[5], cv[6], cv[7]);
    uint32_t c = sel4(q0, q1, XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3);
    uint32_t d = sel4(q0, q1, 0u, 0u, len, flags);
#pragma unroll
    for (int r = 0; r < 7; r++) {
        XFG_B3_GQ(a, b, c, d, sel4(q0, q1, m[0], m[2], m[4], m[6]), sel4(q0, q1, m[1], m[3], m[5], m[7]));
        b = quad_perm<QP_ROT1>(b);
        c = quad_perm<QP_ROT2>(c);
        d = quad_perm<QP_ROT3>(d);
        XFG_B3_GQ(a, b, c, d, sel4(q0, q1, m[8], m[10], m[12], m[14]), sel4(q0, q1, m[9], m[11], m[13], m[15]));
        b = quad_perm<QP_ROT3>(b);
        c = quad_perm<QP_ROT2>(c);
        d = quad_perm<QP_ROT1>(d);
        if (r < 6) XFG_B3_PERMUTE(m);
    }
    return make_uint2(a ^ c, b ^ d);
}
__device__ __forceinline__ uint2 b3_merge_quad(uint32_t m[16], int q) {
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    return b3_compress_quad(iv, m, 64, B3_CHUNK_START | B3_CHUNK_END | B3_ROOT, q);
}
// a wave-uniform compression (every lane holding the same block: the transcript steps) split over each
// quad as above, the eight output words then broadcast to the quad's lanes (DPP quad_perm [k,k,k,k])
__device__ __forceinline__ void b3_compress_uniform(const uint32_t cv[8], uint32_t m[16], uint32_t len, uint32_t flags,
                                                    uint32_t out[8]) {
    const uint2 o = b3_compress_quad(cv, m, len, flags, (int)(threadIdx.x & 3));
    out[0] = quad_perm<0x00>(o.x);
    out[1] = quad_perm<0x55>(o.x);
    out[2] = quad_perm<0xAA>(o.x);
    out[3] = quad_perm<0xFF>(o.x);
    out[4] = quad_perm<0x00>(o.y);
    out[5] = quad_perm<0x55>(o.y);
    out[6] = quad_perm<0xAA>(o.y);
    out[7] = quad_perm<0xFF>(o.y);
}

// ============================================================================ device transcript
// winter-crypto DefaultRandomCoin<Blake3_256> on the device (host twin: host_common.hpp Coin). The
// transcript steps run inside the kernels that produce their inputs: the coefficient, OOD-point and
// FRI alpha draws in the block that computes the Merkle root (tree_top_kernel), the DEEP draws in the
// block that finishes the OOD sums (ood_final_kernel).
__device__ __forceinline__ Digest dev_merge_int(const Digest& seed, u64 v) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = seed.w[i];
    m[8] = (uint32_t)v;
    m[9] = (uint32_t)(v >> 32);
#pragma unroll
    for (int i = 10; i < 16; i++) m[i] = 0;
    return b3_hash_block<0xFC00u>(m, 40);  // words 10..15 are zero
}
// the same for a (seed, v) every lane of the wave holds: four lanes per compression (b3_compress_uniform)
__device__ __forceinline__ Digest dev_merge_int_uniform(const Digest& seed, u64 v) {
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = seed.w[i];
    m[8] = (uint32_t)v;
    m[9] = (uint32_t)(v >> 32);
#pragma unroll
    for (int i = 10; i < 16; i++) m[i] = 0;
    Digest d;
    b3_compress_uniform(iv, m, 40, B3_CHUNK_START | B3_CHUNK_END | B3_ROOT, d.w);
    return d;
}
// acceptance of a drawn candidate (counter, first two LE words): every element < p
struct AcceptP {
    __device__ bool operator()(u64, u64 x, u64 y, int D) const { return x < P && (D == 1 || y < P); }
};
// Coin::draw_e: the first 8 D digest bytes as D LE elements, retried while any is >= p
template <class A = AcceptP>
__device__ __forceinline__ bool dev_draw_e(DevCoin& c, u64* out, int D, A acc = A()) {
    for (int i = 0; i < 1000; i++) {
        const Digest v = dev_merge_int_uniform(c.seed, ++c.counter);
        const u64 x = (u64)v.w[0] | ((u64)v.w[1] << 32), y = (u64)v.w[2] | ((u64)v.w[3] << 32);
        if (acc(c.counter, x, y, D)) {
            out[0] = x;
            out[1] = D == 2 ? y : 0;
            return true;
        }
    }
    return false;
}
__device__ __forceinline__ void dev_reseed(DevCoin& c, const Digest& d) {
    const uint32_t iv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = c.seed.w[i];
        m[8 + i] = d.w[i];
    }
    b3_compress_uniform(iv, m, 64, B3_CHUNK_START | B3_CHUNK_END | B3_ROOT, c.seed.w);
    c.counter = 0;
}
// Blake3_256::hash_elements of cnt <= 128 elements: one chunk of ceil(8 cnt / 64) blocks. Like dev_reseed and
// dev_draw_e, called by a whole wave with the same inputs in every lane (four lanes per compression)
__device__ Digest dev_hash_elems(const u64* e, int cnt) {
    uint32_t cv[8] = {XFG_B3_IV0, XFG_B3_IV1, XFG_B3_IV2, XFG_B3_IV3, XFG_B3_IV4, XFG_B3_IV5, XFG_B3_IV6, XFG_B3_IV7};
    const int len = 8 * cnt, nb = (len + 63) / 64;
    Digest d;
    for (int blk = 0; blk < nb; blk++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int k = 8 * blk + i;
            const u64 v = k < cnt ? e[k] : 0;
            m[2 * i] = (uint32_t)v;
            m[2 * i + 1] = (uint32_t)(v >> 32);
        }
        const bool last = blk == nb - 1;
        const uint32_t flags = (blk == 0 ? B3_CHUNK_START : 0u) | (last ? B3_CHUNK_END | B3_ROOT : 0u);
        uint32_t out[8];
        b3_compress_uniform(cv, m, last ? (uint32_t)(len - 64 * blk) : 64u, flags, out);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            cv[i] = out[i];
            d.w[i] = out[i];
        }
    }
    return d;
}
// k <= 64 consecutive draws of E by one full wave, every lane holding the same coin: lane i hashes
// counter + 1 + i at once, and the accepted candidates in counter order are exactly the draws
// Coin::draw_e makes one after another (a rejected candidate is the one its retry skips). Draw j
// goes to out[j S .. j S + D) (S = stride >= D). If the window holds fewer than k accepted candidates (>= 50
// rejections of probability 2^-32 each) the rest are drawn one at a time after the last accepted.
// The latency is one compression instead of k: these draws sit between two launches of the chain.
template <class A = AcceptP>
__device__ bool wave_draw_e(DevCoin& c, int k, int D, u64* out, int S, A acc = A()) {
    const int lane = threadIdx.x & 63;
    const Digest v = dev_merge_int(c.seed, c.counter + 1 + lane);
    const u64 x = (u64)v.w[0] | ((u64)v.w[1] << 32), y = (u64)v.w[2] | ((u64)v.w[3] << 32);
    const bool ok = acc(c.counter + 1 + lane, x, y, D);
    const u64 mask = __ballot(ok);
    const int idx = __popcll(mask & ((1ULL << lane) - 1));
    if (ok && idx < k) {
        out[idx * S] = x;
        if (D == 2) out[idx * S + 1] = y;
    }
    const int got = __popcll(mask);
    if (got >= k) {
        u64 m = mask;
        for (int i = 1; i < k; i++) m &= m - 1;  // lowest set bit = the k-th accepted candidate
        c.counter += __ffsll((unsigned long long)m);
        return true;
    }
    if (got > 0) c.counter += 64 - __clzll(mask);  // just past the last accepted candidate
    bool all = true;
    for (int j = got; j < k; j++) {
        u64 a[2] = {0, 0};
        all &= dev_draw_e(c, a, D, acc);
        if (lane == 0)
            for (int d = 0; d < D; d++) out[j * S + d] = a[d];
    }
    return all;
}
// one wave (all lanes, uniform) of the block that computed proof b's root: reseed with the root,
// then the draws that follow that commitment in Prover::prove
__device__ void coin_root_step(const CoinStep& cs, int b, const Digest& root) {
    const int D = cs.ext, lane = threadIdx.x;
    DevCoin c = cs.coins[b];
    dev_reseed(c, root);
    bool ok;
    if (cs.kind == CoinStep::COEFFS) {  // 7 transition + 8 boundary composition coefficients
        ok = wave_draw_e(c, 15, D, cs.out + (u64)b * 15 * D, D);
    } else {
        u64 a[2] = {0, 0};
        ok = dev_draw_e(c, a, D);
        if (cs.kind == CoinStep::OOD_POINT) {  // z, and z g; z = 0 leaves no DEEP quotient
            if (a[0] == 0 && a[1] == 0) ok = false;
            if (lane == 0)
                for (int k = 0; k < D; k++) {
                    cs.out[(u64)b * 2 * D + k] = a[k];
                    cs.out[(u64)b * 2 * D + D + k] = gl_mul(a[k], cs.g);
                }
        } else if (lane == 0) {  // FRI layer alpha, stored as alpha * 7^-1 for the fold
            const u64 inv7 = 0x249249246DB6DB6EULL;
            for (int k = 0; k < D; k++) cs.out[(u64)b * D + k] = gl_mul(a[k], inv7);
            if (cs.hist)
                for (int k = 0; k < D; k++) cs.hist[(u64)b * D + k] = a[k];
        }
    }
    if (lane == 0) {
        if (!ok) cs.fail[b] = 1;
        cs.coins[b] = c;
        if (cs.root_out) cs.root_out[b] = root;
    }
}

// ============================================================================ Merkle
// Heap layout per tree: nodes[1] = root, nodes[i] = H(nodes[2i] || nodes[2i+1]), leaf k at L + k
// (MerkleTree::new / build_merkle_nodes, winter-crypto 0.8.3). For the LDE commitments only the
// levels >= log2(beta) are stored (heap [1, 2n)): the 2^log2(beta) leaves of LDE row m (one per
// coset, coset-major layout) form a register-resident subtree whose top is heap node n + m. The
// few leaves / low nodes a proof opens are recomputed from the LDE by open_rows_kernel.

// subtree over the leaves t = T0 .. T0 + 2^LOG - 1 of LDE row m; compile-time recursion keeps
// every intermediate digest in registers. If `local` is non-null the nodes are also written to
// a local heap (slot 1 = top, leaves at 2^LOGB + t).
template <int NC, int LOGB, int LOG, int T0>
__device__ __forceinline__ Digest lde_subtree(const u64* base, u64 n, u64 m, Digest* local) {
    if constexpr (LOG == 0) {
        u64 row[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) row[c] = base[((u64)c * (1 << LOGB) + T0) * n + m];
        Digest d = b3_hash_elems<NC>(row);
        if (local) local[(1 << LOGB) + T0] = d;
        return d;
    } else {
        Digest l = lde_subtree<NC, LOGB, LOG - 1, T0>(base, n, m, local);
        Digest r = lde_subtree<NC, LOGB, LOG - 1, T0 + (1 << (LOG - 1))>(base, n, m, local);
        Digest p = b3_merge(l, r);
        if (local) local[((1 << LOGB) + T0) >> LOG] = p;
        return p;
    }
}

struct Digest2 {
    Digest a, b;
};
// subtrees of two adjacent LDE rows (m, m+1) over cosets T0 .. T0 + 2^LOG - 1, evaluated depth
// first: each leaf pair is loaded (one 16-byte load per column) right before it is hashed, so
// only O(LOGB) digests per row are live
template <int NC, int LOGB, int LOG, int T0>
__device__ __forceinline__ Digest2 pair_subtree(const u64* base, u64 n, u64 m) {
    if constexpr (LOG == 0) {
        u64 r0[NC], r1[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(base + ((u64)c * (1 << LOGB) + T0) * n + m);
            r0[c] = v.x;
            r1[c] = v.y;
        }
        return Digest2{b3_hash_elems<NC>(r0), b3_hash_elems<NC>(r1)};
    } else {
        Digest2 l = pair_subtree<NC, LOGB, LOG - 1, T0>(base, n, m);
        Digest2 r = pair_subtree<NC, LOGB, LOG - 1, T0 + (1 << (LOG - 1))>(base, n, m);
        return Digest2{b3_merge(l.a, r.a), b3_merge(l.b, r.b)};
    }
}

// Block-level continuation of a Merkle level: thread t of a block of T (power of two) threads
// holds the digest of node blockIdx.x * T + t of the level with `count` nodes (heap [count,
// 2 count)). The block merges its T nodes up log2(T) levels through LDS, storing every parent, so
// only count / T nodes are left for launch_tree_top.
// Levels stop once a level has `wmin` nodes per block (lanes of narrower levels would idle).
__device__ __forceinline__ void block_tree_up(Digest d, Digest* nodes, u64 count, Digest* lds, int wmin) {
    const int t = threadIdx.x;
    u64 c = count;
    for (int w = blockDim.x; w > wmin; w >>= 1) {
        lds[t] = d;
        __syncthreads();
        c >>= 1;
        if (t < w / 2) {
            d = b3_merge(lds[2 * t], lds[2 * t + 1]);
            nodes[c + (u64)blockIdx.x * (w / 2) + t] = d;
        }
        __syncthreads();
    }
}

// two consecutive LDE rows per thread: 2 * 2^LOGB leaves, subtree top at level LOGB + 1 =
// heap node n/2 + m/2; then log2(blockDim) levels more in LDS
template <int NC, int LOGB>
__global__ __launch_bounds__(256) void leaves_lde_kernel(const u64* lde, Digest* nodes_all, u64 node_stride,
                                                         int logn, int wmin) {
    __shared__ Digest lds[256];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y;
    const u64 m2 = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // row pair (grid covers n/2 exactly)
    const u64* base = lde + (u64)proof * NC * (1 << LOGB) * n;
    Digest2 d = pair_subtree<NC, LOGB, LOGB, 0>(base, n, 2 * m2);
    Digest top = b3_merge(d.a, d.b);
    Digest* nodes = nodes_all + (u64)proof * node_stride;
    nodes[n / 2 + m2] = top;
    block_tree_up(top, nodes, n / 2, lds, wmin);
}

// one LDE row per thread: the row's 2^LOGB-leaf subtree (top at heap level log2(beta), not stored),
// then through LDS the row-pair level (heap n/2 + m/2) and one more (n/4 + m/4): 256 rows -> 64 nodes
// per block, n/4 left for launch_tree_top. Against leaves_lde_kernel (two rows per thread) a thread
// holds one row and one pending digest per subtree level -- 49-56 instead of 83-105 VGPRs, 8
// instead of 4-5 waves per SIMD -- for the same compressions: the trace leaves 3.3 % faster, the
// composition leaves unchanged (profiles/r05/leaves_row.txt).
template <int NC, int LOGB>
__global__ __launch_bounds__(256) void leaves_row_kernel(const u64* lde, Digest* nodes_all, u64 node_stride,
                                                         int logn) {
    __shared__ Digest lds[256];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, t = threadIdx.x;
    const u64 m = (u64)blockIdx.x * 256 + t;
    const u64* base = lde + (u64)proof * NC * (1 << LOGB) * n;
    Digest d = lde_subtree<NC, LOGB, LOGB, 0>(base, n, m, nullptr);
    Digest* nodes = nodes_all + (u64)proof * node_stride;
    u64 c = n / 2;
    for (int w = 128; w >= 64; w >>= 1, c >>= 1) {
        lds[t] = d;
        __syncthreads();
        if (t < w) {
            d = b3_merge(lds[2 * t], lds[2 * t + 1]);
            nodes[c + (u64)blockIdx.x * w + t] = d;
        }
        __syncthreads();
    }
}

// The same levels for small launch sets (a lone proof: one wave per SIMD, each running the row's
// 2 beta - 1 compressions in sequence): 2^LOGL lanes per row, each the subtree of beta / 2^LOGL cosets,
// merged across the lane group (__shfl_xor, every lane of the group merging at every level), then the
// row-pair level and one more through LDS: 256 / 2^LOGL rows -> a quarter as many nodes per block.
// 2^LOGL times the waves, and a chain of beta / 2^LOGL + log2 beta + 2 compressions instead of 2 beta + 1.
constexpr int LEAF_LANES_LOG = 1;  // 2 lanes per row (4: 42.5 + 40.4 against 31.8 + 27.9 µs, profiles/r06/leaves_small_ab.txt)
template <int LOGB>
constexpr int leaf_lanes_log() { return LOGB < LEAF_LANES_LOG ? LOGB : LEAF_LANES_LOG; }
template <int NC, int LOGB>
__global__ __launch_bounds__(256) void leaves_row2_kernel(const u64* lde, Digest* nodes_all, u64 node_stride,
                                                          int logn) {
    constexpr int LOGL = leaf_lanes_log<LOGB>(), RB = 256 >> LOGL;  // lanes per row (log2), rows per block
    __shared__ Digest lds[RB];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, t = threadIdx.x, h = t & ((1 << LOGL) - 1), rl = t >> LOGL;
    const u64 m = (u64)blockIdx.x * RB + rl;
    const u64* base = lde + (u64)proof * NC * (1 << LOGB) * n + (u64)h * (1 << (LOGB - LOGL)) * n;
    Digest d = lde_subtree<NC, LOGB, LOGB - LOGL, 0>(base, n, m, nullptr);
#pragma unroll
    for (int k = 0; k < LOGL; k++) {
        Digest r;
#pragma unroll
        for (int w = 0; w < 8; w++) r.w[w] = __shfl_xor(d.w[w], 1 << k);
        d = (h >> k) & 1 ? b3_merge(r, d) : b3_merge(d, r);
    }
    Digest* nodes = nodes_all + (u64)proof * node_stride;
    if (h == 0) lds[rl] = d;
    __syncthreads();
    if (t < RB / 2) {
        d = b3_merge(lds[2 * t], lds[2 * t + 1]);
        nodes[n / 2 + (u64)blockIdx.x * (RB / 2) + t] = d;
    }
    __syncthreads();
    if (t < RB / 2) lds[t] = d;
    __syncthreads();
    if (t < RB / 4) nodes[n / 4 + (u64)blockIdx.x * (RB / 4) + t] = b3_merge(lds[2 * t], lds[2 * t + 1]);
}
// openings: recompute the local subtree heaps of selected rows; entry e = proof << logn | m. One
// lane per leaf (coset t of row m, 2^LOGB lanes per entry inside a wave): the leaf, then LOGB
// merge levels with the right child taken from lane l ^ 2^(k-1) -- 1 + LOGB dependent compressions
// per entry instead of the 2^(LOGB+1) - 1 one lane ran in sequence (a lone proof waits on them).
// Every lane of a group merges at every level (no divergence around the shuffles); the lanes with
// t % 2^k == 0 hold level k's nodes and store them to the local heap (slot 1 = top).
template <int NC, int LOGB>
__global__ __launch_bounds__(64) void open_rows_kernel(const u64* lde, const u64* entries, u64 count, Digest* out,
                                                       int logn) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 e = g >> LOGB;
    const int t = (int)(g & ((1 << LOGB) - 1));
    if (e >= count) return;  // whole groups: count is per entry, groups never straddle a wave
    const u64 n = 1ULL << logn, ent = entries[e];
    const u64 proof = ent >> logn, m = ent & (n - 1);
    const u64* base = lde + proof * NC * (1 << LOGB) * n;
    Digest* local = out + e * (2 << LOGB);
    u64 row[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) row[c] = base[((u64)c * (1 << LOGB) + t) * n + m];
    Digest d = b3_hash_elems<NC>(row);
    local[(1 << LOGB) + t] = d;
#pragma unroll
    for (int k = 1; k <= LOGB; k++) {
        Digest r;
#pragma unroll
        for (int w = 0; w < 8; w++) r.w[w] = __shfl_xor(d.w[w], 1 << (k - 1));
        d = b3_merge(d, r);
        if ((t & ((1 << k) - 1)) == 0) local[((1 << LOGB) + t) >> k] = d;
    }
}

#define XFG_LOGB_DISPATCH(KERNEL, NC, logbeta, ...)                                            \
    switch (logbeta) {                                                                          \
        case 1: hipLaunchKernelGGL((KERNEL<NC, 1>), __VA_ARGS__); break;                        \
        case 2: hipLaunchKernelGGL((KERNEL<NC, 2>), __VA_ARGS__); break;                        \
        case 3: hipLaunchKernelGGL((KERNEL<NC, 3>), __VA_ARGS__); break;                        \
        case 4: hipLaunchKernelGGL((KERNEL<NC, 4>), __VA_ARGS__); break;                        \
        default: break;                                                                         \
    }

// in-block Merkle levels continue while a level keeps >= 64 nodes per block (full waves only); the
// narrower levels go to launch_tree_top
static int up_wmin(u64 T) { return (int)std::min<u64>(T, 64); }
u64 launch_leaves_lde(const u64* lde, int nc, Digest* nodes, u64 node_stride, int npoly, int logn, int logbeta,
                      hipStream_t s) {
    const u64 n = 1ULL << logn, T = std::min<u64>(256, n / 2);
    if (n >= 1024 && logbeta >= 1 && (u64)npoly * (n / 256) < 1024) {  // under one wave per SIMD
        const int logl = logbeta < LEAF_LANES_LOG ? logbeta : LEAF_LANES_LOG;
        dim3 g((unsigned)(n >> (8 - logl)), npoly), b(256);
        if (nc == 7) { XFG_LOGB_DISPATCH(leaves_row2_kernel, 7, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        else if (nc == 2) { XFG_LOGB_DISPATCH(leaves_row2_kernel, 2, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        else { XFG_LOGB_DISPATCH(leaves_row2_kernel, 1, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        XFG_CHECK_LAUNCH();
        return n / 4;
    }
    if (n >= 1024) {
        dim3 g((unsigned)(n / 256), npoly), b(256);
        if (nc == 7) { XFG_LOGB_DISPATCH(leaves_row_kernel, 7, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        else if (nc == 2) { XFG_LOGB_DISPATCH(leaves_row_kernel, 2, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        else { XFG_LOGB_DISPATCH(leaves_row_kernel, 1, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
        XFG_CHECK_LAUNCH();
        return n / 4;
    }
    const int wmin = up_wmin(T);
    dim3 g((unsigned)(n / 2 / T), npoly), b((unsigned)T);
    if (nc == 7) { XFG_LOGB_DISPATCH(leaves_lde_kernel, 7, logbeta, g, b, 0, s, lde, nodes, node_stride, logn, wmin) }
    else if (nc == 2) { XFG_LOGB_DISPATCH(leaves_lde_kernel, 2, logbeta, g, b, 0, s, lde, nodes, node_stride, logn, wmin) }
    else { XFG_LOGB_DISPATCH(leaves_lde_kernel, 1, logbeta, g, b, 0, s, lde, nodes, node_stride, logn, wmin) }
    XFG_CHECK_LAUNCH();
    return n / 2 / T * wmin;
}
void launch_open_rows(const u64* lde, int nc, const u64* entries, u64 count, Digest* out, int logn, int logbeta,
                      hipStream_t s) {
    if (!count) return;
    dim3 g((unsigned)(((count << logbeta) + 63) / 64)), b(64);
    if (nc == 7) { XFG_LOGB_DISPATCH(open_rows_kernel, 7, logbeta, g, b, 0, s, lde, entries, count, out, logn) }
    else if (nc == 2) { XFG_LOGB_DISPATCH(open_rows_kernel, 2, logbeta, g, b, 0, s, lde, entries, count, out, logn) }
    else { XFG_LOGB_DISPATCH(open_rows_kernel, 1, logbeta, g, b, 0, s, lde, entries, count, out, logn) }
    XFG_CHECK_LAUNCH();
}

// last levels (count <= 512): one block per tree, four lanes per node (b3_merge_quad), the levels
// through LDS; then the transcript step `cs` on the root
__global__ __launch_bounds__(1024) void tree_top_kernel(Digest* nodes_all, u64 node_stride, u64 count, CoinStep cs) {
    __shared__ Digest lds[256];
    Digest* nodes = nodes_all + (u64)blockIdx.x * node_stride;
    const int tid = threadIdx.x, i = tid >> 2, q = tid & 3;
    for (u64 c = count; c > 1; c >>= 1) {
        const u64 half = c >> 1;
        const bool act = i < (int)half;  // whole quads
        uint2 o = make_uint2(0, 0);
        if (act) {
            const Digest* src = c == count ? nodes + c + 2 * i : lds + 2 * i;
            uint32_t m[16];
#pragma unroll
            for (int w = 0; w < 8; w++) {
                m[w] = src[0].w[w];
                m[8 + w] = src[1].w[w];
            }
            o = b3_merge_quad(m, q);
        }
        __syncthreads();
        if (act) {
            lds[i].w[q] = o.x;
            lds[i].w[4 + q] = o.y;
            nodes[half + i].w[q] = o.x;
            nodes[half + i].w[4 + q] = o.y;
        }
        __syncthreads();
    }
    if (cs.kind != CoinStep::NONE && tid < 64) coin_root_step(cs, blockIdx.x, count > 1 ? lds[0] : nodes[1]);
}
// middle levels: a block merges 512 consecutive nodes of level `count` (two per thread, coalesced)
// and continues through LDS while a level keeps full waves, writing every parent: 64 nodes per block,
// count / 8 remain. (Merging on down to one node per block ran six more levels on one part-filled
// wave each: 13 wave-compressions per block for the work of 8.)
constexpr int TREE_MID_WMIN = 64, TREE_MID_SHRINK = 8;
__global__ __launch_bounds__(256) void tree_mid_kernel(Digest* nodes_all, u64 node_stride, u64 count) {
    __shared__ Digest lds[256];
    Digest* nodes = nodes_all + (u64)blockIdx.y * node_stride;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const Digest d = b3_merge(nodes[count + 2 * i], nodes[count + 2 * i + 1]);
    nodes[count / 2 + i] = d;
    block_tree_up(d, nodes, count / 2, lds, TREE_MID_WMIN);
}
// the same three levels for small launch sets (under one block per CU: a lone proof's trees), four lanes
// per parent (b3_merge_quad): 128 nodes in, 16 out per block, each level's latency about half
__global__ __launch_bounds__(256) void tree_mid4_kernel(Digest* nodes_all, u64 node_stride, u64 count) {
    __shared__ Digest lds[64];
    Digest* nodes = nodes_all + (u64)blockIdx.y * node_stride;
    const int tid = threadIdx.x, i = tid >> 2, q = tid & 3;
    u64 c = count, first = (u64)blockIdx.x * 64;  // level being merged; this block's first parent in it
    for (int w = 64; w >= 16; w >>= 1, c >>= 1, first >>= 1) {
        const bool act = i < w;  // whole quads
        uint2 o = make_uint2(0, 0);
        if (act) {
            const Digest* src = w == 64 ? nodes + c + 2 * (first + i) : lds + 2 * i;
            uint32_t m[16];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                m[k] = src[0].w[k];
                m[8 + k] = src[1].w[k];
            }
            o = b3_merge_quad(m, q);
        }
        __syncthreads();
        if (act) {
            lds[i].w[q] = o.x;
            lds[i].w[4 + q] = o.y;
            Digest* dst = nodes + c / 2 + first + i;
            dst->w[q] = o.x;
            dst->w[4 + q] = o.y;
        }
        __syncthreads();
    }
}
void launch_tree_top(Digest* nodes, u64 node_stride, u64 count, int npoly, hipStream_t s, const CoinStep& cs) {
    while (count > 512) {
        if ((count / 512) * (u64)npoly < 256)
            hipLaunchKernelGGL(tree_mid4_kernel, dim3((unsigned)(count / 128), npoly), dim3(256), 0, s, nodes,
                               node_stride, count);
        else
            hipLaunchKernelGGL(tree_mid_kernel, dim3((unsigned)(count / 512), npoly), dim3(256), 0, s, nodes,
                               node_stride, count);
        count /= TREE_MID_SHRINK;
    }
    if (count > 1 || cs.kind != CoinStep::NONE) {
        int threads = (int)(2 * count);  // four lanes per node of the widest level
        threads = threads < 64 ? 64 : threads;
        hipLaunchKernelGGL(tree_top_kernel, dim3(npoly), dim3(threads), 0, s, nodes, node_stride, count, cs);
    }
    XFG_CHECK_LAUNCH();
}

// FRI layer value at natural index K of a layer stored coset-major (layer 0) or natural
__device__ __forceinline__ u64 layer_at(const u64* base, bool coset_major, int logn, int logbeta, u64 K) {
    if (!coset_major) return base[K];
    u64 t = K & ((1ULL << logbeta) - 1), m = K >> logbeta;
    return base[(t << logn) + m];
}

// FRI layer leaves (hash_values::<H, E, 8> over transpose_slice rows): leaf i = H(values at
// natural indices i + k*rows, k < 8). All leaves are stored (layers are N/8 and smaller).
// E-valued layers are D coordinate planes `comp_stride` elements apart (per proof: D planes)
template <int D>
__global__ __launch_bounds__(256) void fri_leaves_kernel(const u64* vals, u64 val_stride, u64 comp_stride,
                                                         int coset_major, int logn, int logbeta, u64 rows,
                                                         Digest* nodes_all, u64 node_stride, int wmin) {
    __shared__ Digest lds[256];
    const int proof = blockIdx.y;
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // grid covers rows exactly
    const u64* base = vals + (u64)proof * val_stride;
    u64 v[8 * D];
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
        for (int c = 0; c < D; c++)
            v[k * D + c] = layer_at(base + c * comp_stride, coset_major, logn, logbeta, i + (u64)k * rows);
    Digest d = b3_hash_elems<8 * D>(v);
    Digest* nodes = nodes_all + (u64)proof * node_stride;
    nodes[rows + i] = d;
    block_tree_up(d, nodes, rows, lds, wmin);
}
u64 launch_fri_leaves(const u64* vals, u64 val_stride, u64 comp_stride, bool coset_major, int logn, int logbeta,
                      u64 rows, Digest* nodes, u64 node_stride, int npoly, int ext, hipStream_t s) {
    const u64 T = std::min<u64>(256, rows);
    const int wmin = up_wmin(T);
    dim3 g((unsigned)(rows / T), npoly);
    if (ext == 2)
        hipLaunchKernelGGL(fri_leaves_kernel<2>, g, dim3((unsigned)T), 0, s, vals, val_stride, comp_stride,
                           coset_major ? 1 : 0, logn, logbeta, rows, nodes, node_stride, wmin);
    else
        hipLaunchKernelGGL(fri_leaves_kernel<1>, g, dim3((unsigned)T), 0, s, vals, val_stride, comp_stride,
                           coset_major ? 1 : 0, logn, logbeta, rows, nodes, node_stride, wmin);
    XFG_CHECK_LAUNCH();
    return rows / T * wmin;
}

// ============================================================================ AIR
__global__ void trace_gen_kernel(const AirConst* air, u64* trace, int logn) {
    const u64 n = 1ULL << logn;
    const u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const int proof = blockIdx.y;
    if (s >= n) return;
    const AirConst& A = air[proof];
    u64* tr = trace + (u64)proof * 7 * n;
    // src/burn_mint_air.rs:442-476, state column = floor(4 step / n)
    tr[0 * n + s] = A.pub[0];
    tr[1 * n + s] = A.pub[1];
    tr[2 * n + s] = A.pub[2];
    tr[3 * n + s] = A.pub[3];
    tr[4 * n + s] = (4 * s) >> logn;
    tr[5 * n + s] = A.nullifier;
    tr[6 * n + s] = A.commitment;
}
void launch_trace_gen(const AirConst* air, u64* trace, int logn, int npoly, hipStream_t s) {
    u64 n = 1ULL << logn;
    dim3 g((unsigned)((n + 255) / 256), npoly);
    hipLaunchKernelGGL(trace_gen_kernel, g, dim3(256), 0, s, air, trace, logn);
    XFG_CHECK_LAUNCH();
}

struct CeArgs {
    const u64* lde;
    const AirConst* air;
    const u64* coeffs;
    const u64* div;  // [3][2][n]: (x - g^(n-1))/(x^n - 1), 1/(x - 1), 1/(x - g^(n-1)) by (parity, m)
    u64* ce;
    int logn, logbeta;
};
// One thread per constraint-evaluation point i = 2m + par of the CE domain 7*<w_2n>
// (ce_to_lde_blowup = beta/2: CE point i is LDE row i*beta/2, i.e. coset t = par*beta/2, row m).
// Threads walk m fastest inside one parity so the coset-major LDE reads are coalesced.
// The divisor inverses are data independent and come from a per-(n, beta) table.
// D = extension degree of the composition coefficients (1: FieldExtension::None, 2: Quadratic);
// the evaluations are written as D coordinate planes ce[proof][c][nce].
template <int D>
__global__ __launch_bounds__(256) void constraint_eval_kernel(CeArgs a) {
    using F = FE<D>;
    const u64 n = 1ULL << a.logn, nce = 2 * n;
    const int proof = blockIdx.y;
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // grid covers nce exactly
    const u64 par = g >> a.logn, m = g & (n - 1), i = 2 * m + par;
    const AirConst& A = a.air[proof];
    const u64* co = a.coeffs + (u64)proof * 15 * D;
    const u64 beta = 1ULL << a.logbeta;
    const u64* lde = a.lde + (u64)proof * 7 * beta * n;
    const u64 t = par * (beta / 2), mn = (m + 1) & (n - 1);
    u64 cur[7];
#pragma unroll
    for (int c = 0; c < 7; c++) cur[c] = lde[(((u64)c << a.logbeta) + t) * n + m];
    const u64 nxt4 = lde[((4ULL << a.logbeta) + t) * n + mn];
    // divisor inverses loaded with the frame (not next to the multiplies that use them)
    const u64 di = par * n + m;
    const u64 dv0 = a.div[di], dv1 = a.div[nce + di], dv2 = a.div[2 * nce + di];
    // XfgBurnMintAir::evaluate_transition (reference src/burn_mint_air.rs:335-378)
    const u64 std_burn = 8000000ULL, large_burn = 8000000000ULL;
    u64 r[7];
    r[0] = gl_mul(gl_sub(cur[0], std_burn), gl_sub(cur[0], large_burn));
    r[1] = gl_sub(cur[1], cur[0]);
    r[2] = gl_sub(cur[2], A.pub[2] & 0xFFFFFFFFULL);
    r[3] = gl_sub(cur[3], A.pub[3] & 0xFFFFFFFFULL);
    const u64 d = gl_sub(nxt4, cur[4]);
    r[4] = gl_mul(d, gl_sub(d, 1));
    r[5] = gl_sub(cur[5], A.nullifier);
    r[6] = gl_sub(cur[6], A.commitment);
    F tr = F::zero();
#pragma unroll
    for (int c = 0; c < 7; c++) tr = fe_add(tr, fe_mulb(F::load(co + c * D), r[c]));
    // assertions (src/burn_mint_air.rs:380-395): step 0 on columns 0..6, step n-1 on column 4
    const u64 v0[7] = {A.pub[0], A.pub[1], A.pub[2], A.pub[3], 0, A.nullifier, A.commitment};
    F b0 = F::zero();
#pragma unroll
    for (int c = 0; c < 7; c++) b0 = fe_add(b0, fe_mulb(F::load(co + (7 + c) * D), gl_sub(cur[c], v0[c])));
    const F b1 = fe_mulb(F::load(co + 14 * D), gl_sub(cur[4], 3));
    F val = fe_mulb(tr, dv0);
    val = fe_add(val, fe_mulb(b0, dv1));
    val = fe_add(val, fe_mulb(b1, dv2));
#pragma unroll
    for (int c = 0; c < D; c++) a.ce[((u64)proof * D + c) * nce + i] = val.c(c);
}
void launch_constraint_eval(const u64* lde, const AirConst* air, const u64* coeffs, const u64* div, u64* ce, int logn,
                            int logbeta, int npoly, int ext, hipStream_t s) {
    CeArgs a;
    a.lde = lde; a.air = air; a.coeffs = coeffs; a.div = div; a.ce = ce; a.logn = logn; a.logbeta = logbeta;
    u64 nce = 2ULL << logn;
    int threads = nce < 256 ? (int)nce : 256;
    dim3 g((unsigned)(nce / threads), npoly);
    if (ext == 2) hipLaunchKernelGGL(constraint_eval_kernel<2>, g, dim3(threads), 0, s, a);
    else hipLaunchKernelGGL(constraint_eval_kernel<1>, g, dim3(threads), 0, s, a);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ OOD
// Blocks own CHUNK = T * OOD_R consecutive coefficients (T = min(256, n / OOD_R) threads, thread t
// takes j = base + r T + t: coalesced). Per block the 15 partial sums
//   sum_{j in block} T_c[j] z^j, sum T_c[j] (zg)^j (c < 7), sum H[j] z^j
// are stored in `partial` [proof][block][15]: ood_final adds them up, and the DEEP quotient reuses
// them as its per-block carries (no second pass over the coefficients for the block sums).
#define OOD_R 8
static inline int ood_threads(u64 n) { return (int)std::min<u64>(256, n / OOD_R); }

__device__ __forceinline__ u64 shfl_xor_u64(u64 v, int m, int w) {
    u32 lo = __shfl_xor((u32)v, m, w), hi = __shfl_xor((u32)(v >> 32), m, w);
    return (u64)lo | ((u64)hi << 32);
}

template <int D>
__device__ __forceinline__ FE<D> fe_pow(FE<D> b, u64 e) {
    FE<D> r = FE<D>::zero();
    r.a = 1;
    while (e) {
        if (e & 1) r = fe_mul(r, b);
        b = fe_mul(b, b);
        e >>= 1;
    }
    return r;
}
template <int D>
__device__ __forceinline__ FE<D> fe_plane(const u64* planes, u64 plane_stride, u64 j) {  // coordinates from planes
    FE<D> v;
    v.a = planes[j];
    if constexpr (D == 2) v.b = planes[plane_stride + j];
    return v;
}

// zpts [proof][2][D] = (z, z g); coef [proof][7][n] (base); hcoef [proof][D][n];
// partial [proof][block][15][D]
template <int D>
__global__ __launch_bounds__(256) void ood_kernel(const u64* coef, const u64* hcoef, const u64* zpts, u64* partial,
                                                  int logn) {
    using F = FE<D>;
    __shared__ u64 zb[4][D];
    __shared__ u64 red[4][15][D];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, t = threadIdx.x, T = blockDim.x;
    const u64 base = (u64)blockIdx.x * T * OOD_R;
    const F z = F::load(zpts + (u64)proof * 2 * D), zg = F::load(zpts + (u64)proof * 2 * D + D);
    for (int k = t; k < 4; k += T)  // the block's four start powers on four threads (a lone proof waits on them)
        fe_pow(k & 1 ? zg : z, k < 2 ? base : (u64)T).store(zb[k]);
    __syncthreads();
    F pz = fe_mul(F::load(zb[0]), fe_pow(z, (u64)t)), pzg = fe_mul(F::load(zb[1]), fe_pow(zg, (u64)t));
    const F zT = F::load(zb[2]), zgT = F::load(zb[3]);
    const u64* co = coef + (u64)proof * 7 * n;
    const u64* h = hcoef + (u64)proof * D * n;
    F acc[15];
#pragma unroll
    for (int q = 0; q < 15; q++) acc[q] = F::zero();
    // the 8 (7 columns + H) values of index j + T are loaded before the products of index j run:
    // a load next to its multiply would be waited for one at a time (the field primitives are asm
    // statements the scheduler does not move loads across)
    u64 cur[7], nxt[7];
    F hc, hn;
    {
        const u64 j = base + t;
#pragma unroll
        for (int c = 0; c < 7; c++) cur[c] = co[(u64)c * n + j];
        hc = fe_plane<D>(h, n, j);
    }
#pragma unroll
    for (int r = 0; r < OOD_R; r++) {
        if (r + 1 < OOD_R) {
            const u64 j = base + (u64)(r + 1) * T + t;
#pragma unroll
            for (int c = 0; c < 7; c++) nxt[c] = co[(u64)c * n + j];
            hn = fe_plane<D>(h, n, j);
        }
#pragma unroll
        for (int c = 0; c < 7; c++) {
            acc[2 * c] = fe_add(acc[2 * c], fe_mulb(pz, cur[c]));
            acc[2 * c + 1] = fe_add(acc[2 * c + 1], fe_mulb(pzg, cur[c]));
        }
        acc[14] = fe_add(acc[14], fe_mul(hc, pz));
        pz = fe_mul(pz, zT);
        pzg = fe_mul(pzg, zgT);
        if (r + 1 < OOD_R) {  // (the last iteration loaded nothing)
#pragma unroll
            for (int c = 0; c < 7; c++) cur[c] = nxt[c];
            hc = hn;
        }
    }
    // wave reduction, then across the (up to 4) waves
    const int W = T < 64 ? T : 64;
    for (int m = W / 2; m > 0; m >>= 1) {
#pragma unroll
        for (int q = 0; q < 15; q++) {
            acc[q].a = gl_add(acc[q].a, shfl_xor_u64(acc[q].a, m, W));
            if constexpr (D == 2) acc[q].b = gl_add(acc[q].b, shfl_xor_u64(acc[q].b, m, W));
        }
    }
    if ((t & 63) == 0) {
#pragma unroll
        for (int q = 0; q < 15; q++) acc[q].store(red[t >> 6][q]);
    }
    __syncthreads();
    for (int qc = t; qc < 15 * D; qc += T) {  // T may be below 15 D for short traces
        const int q = qc / D, cc = qc % D;
        u64 v = red[0][q][cc];
        for (int w = 1; w < (T + 63) / 64; w++) v = gl_add(v, red[w][q][cc]);
        partial[((u64)proof * gridDim.x + blockIdx.x) * 15 * D + qc] = v;
    }
}
// DEEP coefficients (Prover::prove after the OOD frame), 128 threads for proof b with the frame o[15 D]
// in LDS: wave 0 runs the transcript (reseed with the two element hashes, the 8 draws), wave 1
// meanwhile inverts z (1 / (z g) = (1 / z) g^-1: one inversion)
__device__ void deep_coin_block(const DeepCoinStep& dc, int b, const u64* o, int D) {
    __shared__ u64 ab[8][2];  // a_0..a_6, gamma
    __shared__ E2 zinv;
    __shared__ int ok_s;
    const u64* zb = dc.zpts + (u64)b * 2 * D;
    const E2 z{zb[0], D == 2 ? zb[1] : 0}, zg{zb[D], D == 2 ? zb[D + 1] : 0};
    const bool zz = z.a == 0 && z.b == 0;  // z g == 0 <=> z == 0
    if (threadIdx.x < 64) {
        DevCoin c = dc.coins[b];
        dev_reseed(c, dev_hash_elems(o, 14 * D));  // [T_c(z), T_c(zg)] x 7, coordinates interleaved
        dev_reseed(c, dev_hash_elems(o + 14 * D, D));  // H(z)
        const bool ok = wave_draw_e(c, 8, D, &ab[0][0], 2);
        if (threadIdx.x == 0) {
            dc.coins[b] = c;
            ok_s = ok;
        }
    } else if (threadIdx.x == 64) {
        zinv = zz ? E2{0, 0} : e2_inv(z);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    DeepParams P = {};
    for (int k = 0; k < 7; k++)
        for (int d = 0; d < D; d++) P.a[k][d] = ab[k][d];
    for (int d = 0; d < D; d++) P.gamma[d] = ab[7][d];
    auto put = [](u64* d, E2 v) { d[0] = v.a; d[1] = v.b; };
    auto ood_e = [&](int q) { return E2{o[q * D], D == 2 ? o[q * D + 1] : 0}; };
    put(P.z, z);
    put(P.zg, zg);
    put(P.zinv, zinv);
    put(P.zginv, e2_mulb(zinv, dc.ginv));
    E2 c1 = e2_mul(E2{P.gamma[0], P.gamma[1]}, ood_e(14)), c2{0, 0};
    for (int k = 0; k < 7; k++) {
        const E2 a{P.a[k][0], P.a[k][1]};
        c1 = e2_add(c1, e2_mul(a, ood_e(2 * k)));
        c2 = e2_add(c2, e2_mul(a, ood_e(2 * k + 1)));
    }
    put(P.c1, c1);
    put(P.c2, c2);
    dc.dp[b] = P;
    if (!ok_s || zz) dc.fail[b] = 1;
}
// OOD block partials -> the frame ood[proof][15][D]; then the DEEP draws when dc.coins is set
// The nblk partials of each of the 15 D values are summed by S threads (the most that fit the block), each
// loading 8 partials before it adds them: one thread per value walking all nblk with a load before
// each (asm) add waited for every load in turn -- nblk = 32 round trips at 2^16, 512 at 2^20.
__global__ __launch_bounds__(128) void ood_final_kernel(const u64* partial, int nblk, int d, u64* ood, DeepCoinStep dc) {
    __shared__ u64 o[30];
    __shared__ u64 red[8][30];
    const int proof = blockIdx.x, t = threadIdx.x, nq = 15 * d;
    int S = 1;
    while (nq * S * 2 <= (int)blockDim.x && S < 8) S <<= 1;
    const int q = t % nq, k = t / nq;
    if (k < S) {
        const u64* pp = partial + (u64)proof * nblk * nq + q;
        u64 s = 0;
        for (int b0 = k; b0 < nblk; b0 += 8 * S) {
            u64 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int b = b0 + u * S;
                v[u] = b < nblk ? pp[(u64)b * nq] : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) s = gl_add(s, v[u]);
        }
        red[k][q] = s;
    }
    __syncthreads();
    if (t < nq) {
        u64 s = red[0][t];
        for (int j = 1; j < S; j++) s = gl_add(s, red[j][t]);
        ood[(u64)proof * nq + t] = s;
        o[t] = s;
    }
    if (!dc.coins) return;
    __syncthreads();
    deep_coin_block(dc, proof, o, d);
}
void launch_ood(const u64* coef, const u64* hcoef, const u64* zpts, u64* partial, u64* ood, int logn, int npoly,
                int ext, hipStream_t s, const DeepCoinStep& dc) {
    const u64 n = 1ULL << logn;
    const int T = ood_threads(n), nblk = (int)(n / ((u64)T * OOD_R));
    if (ext == 2)
        hipLaunchKernelGGL(ood_kernel<2>, dim3(nblk, npoly), dim3(T), 0, s, coef, hcoef, zpts, partial, logn);
    else
        hipLaunchKernelGGL(ood_kernel<1>, dim3(nblk, npoly), dim3(T), 0, s, coef, hcoef, zpts, partial, logn);
    hipLaunchKernelGGL(ood_final_kernel, dim3(npoly), dim3(dc.coins ? 128 : 64), 0, s, partial, nblk, ext, ood, dc);
    XFG_CHECK_LAUNCH();
}
u64 ood_partial_count(int logn) {
    const u64 n = 1ULL << logn;
    return n / ((u64)ood_threads(n) * OOD_R);
}

// ============================================================================ DEEP
// DEEP quotient in coefficient form: P1_j = sum a_c T_c[j] + gamma H[j] - [j==0] c1,
// P2_j = sum a_c T_c[j] - [j==0] c2; d_k = q1_k + q2_k with the synthetic-division recurrences
//   q1_k = P1_{k+1} + z q1_{k+1},  q2_k = P2_{k+1} + zg q2_{k+1},  q_{n-1} = 0.
// Same block chunking as the OOD kernel. Block b's entry carry q_e (e = last index of the block)
// is z^-(e+1) * sum_{j > e} P_j z^j, a weighted suffix sum of the OOD block partials
// (deep_carry_kernel). Inside a block every thread owns OOD_R consecutive indices: a backward
// Horner pass gives its chunk map Q_out = L + z^R Q_in, a suffix scan over threads with the
// uniform multiplier z^R gives each thread's Q_in, and a second backward pass writes d_k.
// All of it in E (extension degree D): coefficients, z and the output planes deep[proof][c][n].
template <int D>
__global__ __launch_bounds__(1024) void deep_carry_kernel(const u64* partial, const DeepParams* dp, u64* carry,
                                                          int nblk, int logch) {
    using F = FE<D>;
    __shared__ u64 S1[1024][D], S2[1024][D];
    const int proof = blockIdx.x, b = threadIdx.x;
    const DeepParams& P = dp[proof];
    F b1 = F::zero(), b2 = F::zero();
    if (b < nblk) {
        const u64* pp = partial + ((u64)proof * nblk + b) * 15 * D;
        F t1 = F::zero(), t2 = F::zero();
#pragma unroll
        for (int c = 0; c < 7; c++) {
            const F a = F::load(P.a[c]);
            t1 = fe_add(t1, fe_mul(a, F::load(pp + 2 * c * D)));
            t2 = fe_add(t2, fe_mul(a, F::load(pp + (2 * c + 1) * D)));
        }
        b1 = fe_add(t1, fe_mul(F::load(P.gamma), F::load(pp + 14 * D)));
        b2 = t2;
        if (b == 0) {
            b1 = fe_sub(b1, F::load(P.c1));
            b2 = fe_sub(b2, F::load(P.c2));
        }
    }
    b1.store(S1[b]);
    b2.store(S2[b]);
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {  // inclusive suffix sums
        F v1 = F::load(S1[b]), v2 = F::load(S2[b]);
        if (b + off < (int)blockDim.x) {
            v1 = fe_add(v1, F::load(S1[b + off]));
            v2 = fe_add(v2, F::load(S2[b + off]));
        }
        __syncthreads();
        v1.store(S1[b]);
        v2.store(S2[b]);
        __syncthreads();
    }
    if (b < nblk) {
        const u64 e = (u64)(b + 1) << logch;  // carry into block b: z^-e * sum over blocks after b
        const F x1 = b + 1 < nblk ? F::load(S1[b + 1]) : F::zero();
        const F x2 = b + 1 < nblk ? F::load(S2[b + 1]) : F::zero();
        fe_mul(x1, fe_pow(F::load(P.zinv), e)).store(carry + (((u64)proof * nblk + b) * 2) * D);
        fe_mul(x2, fe_pow(F::load(P.zginv), e)).store(carry + (((u64)proof * nblk + b) * 2 + 1) * D);
    }
}
__device__ __forceinline__ int dpad(int i) { return i + i / OOD_R; }  // chunk stride R+1: no bank pile-up
template <int D>
__global__ __launch_bounds__(256) void deep_final_kernel(const u64* coef, const u64* hcoef, const DeepParams* dp,
                                                         const u64* carry, u64* deep, int logn) {
    using F = FE<D>;
    constexpr int R = OOD_R, CHMAX = 256 * OOD_R, PADN = CHMAX + CHMAX / R;
    __shared__ u64 s1[D][PADN], s2[D][PADN];
    __shared__ u64 S1[256][D], S2[256][D];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, t = threadIdx.x, T = blockDim.x;
    const u64 base = (u64)blockIdx.x * T * R;
    const DeepParams& P = dp[proof];
    const F z = F::load(P.z), zg = F::load(P.zg), gam = F::load(P.gamma);
    F ac[7];
#pragma unroll
    for (int c = 0; c < 7; c++) ac[c] = F::load(P.a[c]);
    const u64* co = coef + (u64)proof * 7 * n;
    const u64* h = hcoef + (u64)proof * D * n;
    auto lds_ld = [&](u64 (*arr)[PADN], int k) {
        F v;
        v.a = arr[0][k];
        if constexpr (D == 2) v.b = arr[1][k];
        return v;
    };
    auto lds_st = [&](u64 (*arr)[PADN], int k, F v) {
        arr[0][k] = v.a;
        if constexpr (D == 2) arr[1][k] = v.b;
    };
    // 1. P1, P2 (coalesced reads) into LDS
#pragma unroll 2
    for (int r = 0; r < R; r++) {
        const int li = r * T + t;
        const u64 j = base + li;
        F sacc = F::zero();
#pragma unroll
        for (int c = 0; c < 7; c++) sacc = fe_add(sacc, fe_mulb(ac[c], co[(u64)c * n + j]));
        F p1 = fe_add(sacc, fe_mul(gam, fe_plane<D>(h, n, j))), p2 = sacc;
        if (j == 0) {
            p1 = fe_sub(p1, F::load(P.c1));
            p2 = fe_sub(p2, F::load(P.c2));
        }
        lds_st(s1, dpad(li), p1);
        lds_st(s2, dpad(li), p2);
    }
    __syncthreads();
    // 2. chunk maps: L = sum_i z^i P_{a+i}
    const int a = t * R;
    F L1 = F::zero(), L2 = F::zero();
#pragma unroll
    for (int i = R - 1; i >= 0; i--) {
        L1 = fe_add(lds_ld(s1, dpad(a + i)), fe_mul(z, L1));
        L2 = fe_add(lds_ld(s2, dpad(a + i)), fe_mul(zg, L2));
    }
    // 3. suffix scan over threads, multiplier w = z^R; the block carry enters through the last thread
    F w1 = z, w2 = zg;
#pragma unroll
    for (int i = 1; i < R; i <<= 1) {
        w1 = fe_mul(w1, w1);
        w2 = fe_mul(w2, w2);
    }
    const F cin1 = F::load(carry + (((u64)proof * gridDim.x + blockIdx.x) * 2) * D);
    const F cin2 = F::load(carry + (((u64)proof * gridDim.x + blockIdx.x) * 2 + 1) * D);
    if (t == T - 1) {
        L1 = fe_add(L1, fe_mul(w1, cin1));
        L2 = fe_add(L2, fe_mul(w2, cin2));
    }
    L1.store(S1[t]);
    L2.store(S2[t]);
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {
        F v1 = F::load(S1[t]), v2 = F::load(S2[t]);
        if (t + off < T) {
            v1 = fe_add(v1, fe_mul(w1, F::load(S1[t + off])));
            v2 = fe_add(v2, fe_mul(w2, F::load(S2[t + off])));
        }
        __syncthreads();
        v1.store(S1[t]);
        v2.store(S2[t]);
        __syncthreads();
        w1 = fe_mul(w1, w1);
        w2 = fe_mul(w2, w2);
    }
    F q1 = t + 1 < T ? F::load(S1[t + 1]) : cin1, q2 = t + 1 < T ? F::load(S2[t + 1]) : cin2;
    // 4. backward pass over the chunk: d_k = q1_k + q2_k, then step to k - 1
#pragma unroll
    for (int i = R - 1; i >= 0; i--) {
        const int k = dpad(a + i);
        const F p1 = lds_ld(s1, k), p2 = lds_ld(s2, k);
        lds_st(s1, k, fe_add(q1, q2));
        q1 = fe_add(p1, fe_mul(z, q1));
        q2 = fe_add(p2, fe_mul(zg, q2));
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < D; c++) {
        u64* out = deep + ((u64)proof * D + c) * n + base;
#pragma unroll
        for (int r = 0; r < R; r++) out[r * T + t] = s1[c][dpad(r * T + t)];
    }
}
void launch_deep(const u64* coef, const u64* hcoef, const DeepParams* dp, const u64* partial, u64* carry, u64* deep,
                 int logn, int npoly, int ext, hipStream_t s) {
    const u64 n = 1ULL << logn;
    const int T = ood_threads(n), nblk = (int)(n / ((u64)T * OOD_R));
    int logch = 0;
    while ((1ULL << logch) < (u64)T * OOD_R) logch++;
    int ct = 64;
    while (ct < nblk) ct <<= 1;  // nblk <= 1024 (n <= 2^21, 2048 coefficients per block)
    if (ext == 2) {
        hipLaunchKernelGGL(deep_carry_kernel<2>, dim3(npoly), dim3(ct), 0, s, partial, dp, carry, nblk, logch);
        hipLaunchKernelGGL(deep_final_kernel<2>, dim3(nblk, npoly), dim3(T), 0, s, coef, hcoef, dp, carry, deep, logn);
    } else {
        hipLaunchKernelGGL(deep_carry_kernel<1>, dim3(npoly), dim3(ct), 0, s, partial, dp, carry, nblk, logch);
        hipLaunchKernelGGL(deep_final_kernel<1>, dim3(nblk, npoly), dim3(T), 0, s, coef, hcoef, dp, carry, deep, logn);
    }
    XFG_CHECK_LAUNCH();
}

// ============================================================================ FRI fold
// apply_drp for folding factor 8 with Winterfell's constant domain offset 7 on every layer:
// row i = {v_k at 7 w_D^i zeta^k}; c = iDFT_8(v)/8 ; result = sum_j c_j (alpha / (7 w_D^i))^j
struct FoldArgs {
    const u64* vals;
    u64 val_stride, comp_stride;
    int coset_major, logn, logbeta;
    u64 rows;
    int logD;
    const u64* alpha7;  // [proof][D]: alpha * 7^-1
    u64* out;           // [proof][D][rows]
    u64 out_stride;
    Tables T;
};
template <int D>
__global__ __launch_bounds__(256) void fri_fold_kernel(FoldArgs a) {
    using F = FE<D>;
    const int proof = blockIdx.y;
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.rows) return;
    const u64* base = a.vals + (u64)proof * a.val_stride;
    // the size-8 inverse DFT per coordinate (base-field twiddles w_8^-k = powers of two: shifts),
    // natural order in and out, outputs canonicalised for the Horner adds
    u64 c[D][8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u64 K = i + (u64)k * a.rows;
        c[0][k] = layer_at(base, a.coset_major, a.logn, a.logbeta, K);
        if constexpr (D == 2) c[1][k] = layer_at(base + a.comp_stride, a.coset_major, a.logn, a.logbeta, K);
    }
    F v[8];
#pragma unroll
    for (int d = 0; d < D; d++) {
        dft_reg<3, true>(c[d]);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (d == 0) v[k].a = canon(c[d][k]);
            if constexpr (D == 2) if (d == 1) v[k].b = canon(c[d][k]);
        }
    }
    // y = alpha * 7^-1 * w_D^-i ; Horner
    const F y = fe_mulb(F::load(a.alpha7 + (u64)proof * D), tw_ipow(a.T, a.logD, i));
    F r = v[7];
#pragma unroll
    for (int j = 6; j >= 0; j--) r = fe_add(fe_mul(r, y), v[j]);
    // 1/8 = 2^-3 = 2^189 = -2^93
#pragma unroll
    for (int d = 0; d < D; d++) {
        const u64 x = gl_neg(mul_pow2<93>(r.c(d)));
        if (d == 0) r.a = x;
        if constexpr (D == 2) if (d == 1) r.b = x;
    }
#pragma unroll
    for (int c = 0; c < D; c++) a.out[((u64)proof * D + c) * a.out_stride + i] = r.c(c);
}
void launch_fri_fold(const u64* vals, u64 val_stride, u64 comp_stride, bool coset_major, int logn, int logbeta,
                     u64 rows, int logD, const u64* alpha7, u64* out, u64 out_stride, const Tables& T, int npoly,
                     int ext, hipStream_t s) {
    FoldArgs a;
    a.vals = vals; a.val_stride = val_stride; a.comp_stride = comp_stride; a.coset_major = coset_major ? 1 : 0;
    a.logn = logn; a.logbeta = logbeta; a.rows = rows; a.logD = logD; a.alpha7 = alpha7; a.out = out;
    a.out_stride = out_stride;
    a.T = T;
    int threads = rows < 256 ? (int)rows : 256;
    dim3 g((unsigned)((rows + threads - 1) / threads), npoly);
    if (ext == 2) hipLaunchKernelGGL(fri_fold_kernel<2>, g, dim3(threads), 0, s, a);
    else hipLaunchKernelGGL(fri_fold_kernel<1>, g, dim3(threads), 0, s, a);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ transcript self test
// AcceptP plus forced rejections: candidate counter c in [1, 256] is rejected when bit c - 1 of
// rej[4] is set (exercises wave_draw_e's window bookkeeping and its one-at-a-time fallback)
struct AcceptForced {
    const u64* rej;
    __device__ bool operator()(u64 ctr, u64 x, u64 y, int D) const {
        const bool forced = ctr >= 1 && ctr <= 256 && ((rej[(ctr - 1) >> 6] >> ((ctr - 1) & 63)) & 1);
        return !forced && AcceptP()(ctr, x, y, D);
    }
};
__global__ __launch_bounds__(64) void coin_draw_test_kernel(DevCoin c0, int k, int D, const u64* rej, u64* out_wave,
                                                            u64* out_seq, u64* ctr, int* ok) {
    const AcceptForced acc{rej};
    DevCoin c = c0;
    const bool okw = wave_draw_e(c, k, D, out_wave, 2, acc);
    DevCoin q = c0;
    bool oks = true;
    for (int j = 0; j < k; j++) {
        u64 a[2] = {0, 0};
        oks &= dev_draw_e(q, a, D, acc);
        if (threadIdx.x == 0) {
            out_seq[2 * j] = a[0];
            out_seq[2 * j + 1] = a[1];
        }
    }
    if (threadIdx.x == 0) {
        ctr[0] = c.counter;
        ctr[1] = q.counter;
        ok[0] = okw;
        ok[1] = oks;
    }
}
void launch_coin_draw_test(const DevCoin& c0, int k, int ext, const u64* rej, u64* out_wave, u64* out_seq, u64* ctr,
                           int* ok, hipStream_t s) {
    hipLaunchKernelGGL(coin_draw_test_kernel, dim3(1), dim3(64), 0, s, c0, k, ext, rej, out_wave, out_seq, ctr, ok);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ gathers
// all of a unit's opening gathers in one launch: thread i of the grid serves element i - first[k] of
// segment k (the segments are laid end to end in index order; at most GatherSet::MAX of them)
__global__ void gather_set_kernel(GatherSet g, const u64* idx) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.first[g.nseg]) return;
    int k = 0;
    while (i >= g.first[k + 1]) k++;
    const u64 src = idx[i];
    if (g.digest[k]) {
        const Digest* s = (const Digest*)g.src[k];
        ((Digest*)g.dst[k])[i - g.first[k]] = s[src];
    } else {
        ((u64*)g.dst[k])[i - g.first[k]] = ((const u64*)g.src[k])[src];
    }
}
void launch_gather_set(const GatherSet& g, const u64* idx, hipStream_t s) {
    const u64 total = g.first[g.nseg];
    if (!total) return;
    hipLaunchKernelGGL(gather_set_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, g, idx);
    XFG_CHECK_LAUNCH();
}

// one segment per blockIdx.y, grid-stride over its words
__global__ void pack_kernel(PackSet p, u32* dst) {
    const int k = blockIdx.y;
    const u32* src = (const u32*)p.src[k];
    u32* out = dst + p.off[k];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < p.words[k]; i += (u64)gridDim.x * blockDim.x)
        out[i] = src[i];
}
void launch_pack(const PackSet& p, void* dst, hipStream_t s) {
    u64 most = 0;
    for (int k = 0; k < p.nseg; k++) most = std::max(most, p.words[k]);
    if (!most) return;
    const unsigned bx = (unsigned)std::min<u64>(32, (most + 255) / 256);
    hipLaunchKernelGGL(pack_kernel, dim3(bx, p.nseg), dim3(256), 0, s, p, (u32*)dst);
    XFG_CHECK_LAUNCH();
}

}  // namespace xfg
