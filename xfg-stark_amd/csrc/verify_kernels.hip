// Batched verification on the GPU (gfx950): the Merkle openings and the per-query DEEP / FRI /
// remainder checks of many burn proofs at once. The host replays each transcript and lays the work
// out as flat task lists (verifier.cpp plan_proof); see xfg_verify_batch_gpu in prover.hip.
// Replaces the serial BatchBurnMintVerifier loops of the reference (src/burn_mint_verifier.rs:
// 326-338, 386-408), each of which runs winterfell::verify on the CPU.
#include "verifier.hpp"

namespace xfg {

// proof bytes are not 8-aligned inside the blob: assemble words from bytes
__device__ __forceinline__ u64 ld_u64(const uint8_t* p) {
    u64 v = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) v |= (u64)p[i] << (8 * i);
    return v;
}
__device__ __forceinline__ E2 ld_e(const uint8_t* p, int de) { return de == 2 ? E2{ld_u64(p), ld_u64(p + 8)} : E2{ld_u64(p), 0}; }

template <int K>
__device__ __forceinline__ Digest hash_words(const uint8_t* p) {
    u64 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = ld_u64(p + 8 * k);
    return b3_hash_elems<K>(v);
}
__device__ Digest hash_row(const uint8_t* p, uint32_t words) {
    switch (words) {  // trace row 7, constraint value 1 / 2, FRI row 8 / 16
        case 1: return hash_words<1>(p);
        case 2: return hash_words<2>(p);
        case 7: return hash_words<7>(p);
        case 8: return hash_words<8>(p);
        default: return hash_words<16>(p);
    }
}
__device__ __forceinline__ Digest ld_digest(const uint8_t* p) {
    Digest d;
#pragma unroll
    for (int w = 0; w < 8; w++)
        d.w[w] = (uint32_t)p[4 * w] | ((uint32_t)p[4 * w + 1] << 8) | ((uint32_t)p[4 * w + 2] << 16) |
                 ((uint32_t)p[4 * w + 3] << 24);
    return d;
}

// exclusive prefix count of `f` over the workgroup's 256 threads (4 waves), and the total
__device__ __forceinline__ int block_scan(bool f, int* wsum, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long m = __ballot(f);
    const int pre = __popcll(m & ((1ULL << lane) - 1));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int base = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        base += k < w ? wsum[k] : 0;
        total += wsum[k];
    }
    __syncthreads();
    return base + pre;
}

// One batch Merkle opening per workgroup: BatchMerkleProof::get_root (winter-crypto 0.8.3, the
// opening plan_batch_opening emits) recomputed in place. Thread i hashes opened row i (rows sorted
// by leaf index); the distinct leaf pairs take their missing leaf from node vector j (j = the pair's
// position); then, level by level, the entry at position j of the current sorted list merges with
// its right neighbour when that is its sibling, else takes its sibling from vector j; the survivors
// are compacted (block scan) and climb one level. The opening is valid when every vector holds the
// nodes the walk takes (nodes past them are ignored, as winter-crypto 0.8's get_root ignores them:
// verifier.cpp merkle_symbolic) and the root equals the commitment; else flags[proof] |= bit.
__global__ __launch_bounds__(256) void vtree_kernel(const uint8_t* blob, const VTree* trees, const VTreeLeaf* tleaves,
                                                    const VVec* vecs, uint32_t* flags) {
    __shared__ Digest leaf[512];
    __shared__ Digest dg[2][256];
    __shared__ u64 hx[2][256];
    __shared__ u64 sidx[256];
    __shared__ uint8_t have[512];
    __shared__ int wsum[4];
    __shared__ int bad;
    const VTree T = trees[blockIdx.x];
    const int i = threadIdx.x;
    const u64 L = 1ULL << T.depth;
    if (i == 0) bad = 0;
    // the vector this thread's position consumes from, and how many nodes it has taken
    VVec vec{0, 0, 0};
    if (i < (int)T.nvec) vec = vecs[T.vec0 + i];
    uint32_t used = 0;
    auto take = [&](Digest& out) {
        if (used >= vec.cnt) {
            bad = 1;
            out = Digest{};
            return;
        }
        out = ld_digest(blob + vec.off + 32 * (u64)used);
        used++;
    };
    u64 idx = 0;
    Digest ld{};
    const bool opened = i < (int)T.nidx;
    if (opened) {
        const VTreeLeaf lf = tleaves[T.leaf0 + i];
        idx = lf.index;
        ld = hash_row(blob + lf.row_off, T.words);
        sidx[i] = idx;
    }
    have[i] = 0;
    have[i + 256] = 0;
    __syncthreads();
    // leaf pairs: thread i's pair position = number of pair starts before it (minus one if it is the
    // right leaf of a pair whose left leaf is opened too)
    const bool start = opened && (i == 0 || (sidx[i - 1] >> 1) != (idx >> 1));
    int npairs;
    const int pp = block_scan(start, wsum, npairs) - (opened && !start ? 1 : 0);
    if (opened) {
        leaf[2 * pp + (idx & 1)] = ld;
        have[2 * pp + (idx & 1)] = 1;
        if (start) hx[0][pp] = (L + (idx & ~1ULL)) >> 1;
    }
    if (i == 0 && (int)T.nvec != npairs) bad = 1;
    __syncthreads();
    if (i < npairs) {
        Digest l = leaf[2 * i], r = leaf[2 * i + 1];
        if (!have[2 * i]) take(l);
        if (!have[2 * i + 1]) take(r);
        dg[0][i] = b3_merge(l, r);
    }
    __syncthreads();
    int nn = npairs, cb = 0;
    for (unsigned lvl = 1; lvl < T.depth; lvl++) {
        const bool act = i < nn;
        const u64 h = act ? hx[cb][i] : 0;
        const bool left = act && !(h & 1) && i + 1 < nn && hx[cb][i + 1] == h + 1;
        const bool right = act && (h & 1) && i > 0 && hx[cb][i - 1] == h - 1;
        Digest par{};
        if (act && !right) {  // one merge call site: (own, right neighbour) or (own, vector node) in order
            Digest x = dg[cb][i], y;
            if (left) {
                y = dg[cb][i + 1];
            } else {
                take(y);
                if (h & 1) {
                    const Digest t = x;
                    x = y;
                    y = t;
                }
            }
            par = b3_merge(x, y);
        }
        int total;
        const int m = block_scan(act && !right, wsum, total);
        if (act && !right) {
            hx[cb ^ 1][m] = h >> 1;
            dg[cb ^ 1][m] = par;
        }
        __syncthreads();
        nn = total;
        cb ^= 1;
    }
    __syncthreads();
    if (i == 0) {
        const Digest root = ld_digest(blob + T.root_off);
        bool ok = !bad && nn == 1 && hx[cb][0] == 1;
        for (int w = 0; w < 8; w++) ok = ok && dg[cb][0].w[w] == root.w[w];
        if (!ok) atomicOr(&flags[T.proof], T.bit);
    }
}

// apply_drp of one row: iDFT_8 on the coset x<w_8> (per coordinate), evaluate at alpha
__device__ E2 vfold(const E2 v[8], u64 x, E2 alpha) {
    const u64 winv = gl_inv(gl_root(3)), inv8 = gl_inv(8);
    E2 c[8];
    for (int k = 0; k < 8; k++) {
        E2 s{0, 0};
        u64 wk = gl_pow(winv, (u64)k), p = 1;
        for (int j = 0; j < 8; j++) {
            s = e2_add(s, e2_mulb(v[j], p));
            p = gl_mul(p, wk);
        }
        c[k] = e2_mulb(s, inv8);
    }
    const E2 t = e2_mulb(alpha, gl_inv(x));
    E2 r{0, 0};
    for (int k = 7; k >= 0; k--) r = e2_add(e2_mul(r, t), c[k]);
    return r;
}

// one thread per (proof, query): DEEP value at the query point, then every FRI layer's opened value
// against the running fold, then the remainder polynomial; failures set bits of flags[proof]
// (bit l: layer l folding, bit 31: remainder)
__global__ __launch_bounds__(64) void vfield_kernel(const uint8_t* blob, const VFieldProof* fp, const VFieldQuery* fq,
                                                    u64 nq, uint32_t* flags) {
    const u64 qi = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    const VFieldQuery& Q = fq[qi];
    const VFieldProof& P = fp[Q.proof];
    const int de = (int)P.de;
    const u64 N = 1ULL << P.logN;
    E2 x = e2(gl_mul(GEN, gl_pow(gl_root(P.logN), Q.pos)));
    E2 s1{0, 0}, s2{0, 0};
    for (int c = 0; c < 7; c++) {
        const E2 tx = e2(ld_u64(blob + Q.trace_off + 8 * c));
        s1 = e2_add(s1, e2_mul(P.dc[c], e2_sub(tx, P.ood[2 * c])));
        s2 = e2_add(s2, e2_mul(P.dc[c], e2_sub(tx, P.ood[2 * c + 1])));
    }
    const E2 izx = e2_inv(e2_sub(x, P.z)), izgx = e2_inv(e2_sub(x, P.zg));
    E2 ev = e2_add(e2_mul(s1, izx), e2_mul(s2, izgx));
    ev = e2_add(ev, e2_mul(e2_mul(P.gam, e2_sub(ld_e(blob + Q.cons_off, de), P.hz)), izx));
    u64 D = N, p = Q.pos;
    uint32_t bad = 0;
    for (uint32_t l = 0; l < P.nl; l++) {
        const u64 rows = D / 8, i = p & (rows - 1), k = p / rows;
        const uint8_t* row = blob + Q.row_off[l];
        E2 v[8];
        for (int j = 0; j < 8; j++) v[j] = ld_e(row + 8 * de * j, de);
        if (!e2_eq(v[k], ev)) bad |= 1u << l;
        int logD = 0;
        while ((1ULL << logD) < D) logD++;
        ev = vfold(v, gl_mul(GEN, gl_pow(gl_root(logD), i)), P.falpha[l]);
        p = i;
        D = rows;
    }
    int logD = 0;
    while ((1ULL << logD) < D) logD++;
    const E2 xr = e2(gl_mul(GEN, gl_pow(gl_root(logD), p)));
    E2 r{0, 0};
    for (uint32_t k = P.rem_len; k-- > 0;) r = e2_add(e2_mul(r, xr), ld_e(blob + P.rem_off + 8 * de * k, de));
    if (!e2_eq(r, ev)) bad |= 1u << 31;
    if (bad) atomicOr(&flags[Q.proof], bad);
}

static unsigned blocks_for(u64 n, unsigned t) { return (unsigned)((n + t - 1) / t); }

void launch_verify(const uint8_t* blob, const VTree* trees, u64 ntrees, const VTreeLeaf* tleaves, const VVec* vecs,
                   const VFieldProof* fp, const VFieldQuery* fq, u64 nq, uint32_t* flags, hipStream_t s) {
    if (ntrees) hipLaunchKernelGGL(vtree_kernel, dim3((unsigned)ntrees), dim3(256), 0, s, blob, trees, tleaves, vecs, flags);
    if (nq) hipLaunchKernelGGL(vfield_kernel, dim3(blocks_for(nq, 64)), dim3(64), 0, s, blob, fp, fq, nq, flags);
    (void)hipGetLastError();
}

}  // namespace xfg
