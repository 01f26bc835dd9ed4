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

// two consecutive LDE rows per thread: 2 * 2^LOGB leaves, subtree top at level LOGB + 1 =
// heap node n/2 + m/2
template <int NC, int LOGB>
__global__ __launch_bounds__(256) void leaves_lde_kernel(const u64* lde, Digest* nodes_all, u64 node_stride,
                                                         int logn) {
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y;
    const u64 m2 = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // row pair
    if (2 * m2 >= n) return;
    const u64* base = lde + (u64)proof * NC * (1 << LOGB) * n;
    Digest2 d = pair_subtree<NC, LOGB, LOGB, 0>(base, n, 2 * m2);
    nodes_all[(u64)proof * node_stride + n / 2 + m2] = b3_merge(d.a, d.b);
}

// openings: recompute the local subtree heaps of selected rows; entry e = proof << logn | m
template <int NC, int LOGB>
__global__ __launch_bounds__(64) void open_rows_kernel(const u64* lde, const u64* entries, u64 count, Digest* out,
                                                       int logn) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    const u64 n = 1ULL << logn, ent = entries[e];
    const u64 proof = ent >> logn, m = ent & (n - 1);
    const u64* base = lde + proof * NC * (1 << LOGB) * n;
    lde_subtree<NC, LOGB, LOGB, 0>(base, n, m, out + e * (2 << LOGB));
}

#define XFG_LOGB_DISPATCH(KERNEL, NC, logbeta, ...)                                            \
    switch (logbeta) {                                                                          \
        case 1: hipLaunchKernelGGL((KERNEL<NC, 1>), __VA_ARGS__); break;                        \
        case 2: hipLaunchKernelGGL((KERNEL<NC, 2>), __VA_ARGS__); break;                        \
        case 3: hipLaunchKernelGGL((KERNEL<NC, 3>), __VA_ARGS__); break;                        \
        case 4: hipLaunchKernelGGL((KERNEL<NC, 4>), __VA_ARGS__); break;                        \
        default: break;                                                                         \
    }

void launch_leaves_lde(const u64* lde, int nc, Digest* nodes, u64 node_stride, int npoly, int logn, int logbeta,
                       hipStream_t s) {
    u64 n = 1ULL << logn;
    dim3 g((unsigned)((n / 2 + 255) / 256), npoly), b(256);
    if (nc == 7) { XFG_LOGB_DISPATCH(leaves_lde_kernel, 7, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
    else { XFG_LOGB_DISPATCH(leaves_lde_kernel, 1, logbeta, g, b, 0, s, lde, nodes, node_stride, logn) }
    XFG_CHECK_LAUNCH();
}
void launch_open_rows(const u64* lde, int nc, const u64* entries, u64 count, Digest* out, int logn, int logbeta,
                      hipStream_t s) {
    if (!count) return;
    dim3 g((unsigned)((count + 63) / 64)), b(64);
    if (nc == 7) { XFG_LOGB_DISPATCH(open_rows_kernel, 7, logbeta, g, b, 0, s, lde, entries, count, out, logn) }
    else { XFG_LOGB_DISPATCH(open_rows_kernel, 1, logbeta, g, b, 0, s, lde, entries, count, out, logn) }
    XFG_CHECK_LAUNCH();
}

// one thread per node of level `count >> H`: merges its 2^H descendants at level `count`
// (heap [count, 2 count)) in registers and writes the H levels above them
template <int H>
__device__ __forceinline__ Digest up_subtree(const Digest* src, Digest* nodes, u64 first, int lvl_from_top) {
    (void)lvl_from_top;
    if constexpr (H == 0) {
        return src[0];
    } else {
        Digest l = up_subtree<H - 1>(src, nodes, first, 0);
        Digest r = up_subtree<H - 1>(src + (1 << (H - 1)), nodes, first + (1ULL << (H - 1)), 0);
        Digest p = b3_merge(l, r);
        nodes[first >> H] = p;
        return p;
    }
}
template <int H>
__global__ __launch_bounds__(256) void tree_up_kernel(Digest* nodes_all, u64 node_stride, u64 count) {
    const u64 idx = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (count >> H)) return;
    Digest* nodes = nodes_all + (u64)blockIdx.y * node_stride;
    const u64 first = count + (idx << H);
    Digest ch[1 << H];
#pragma unroll
    for (int k = 0; k < (1 << H); k++) ch[k] = nodes[first + k];
    up_subtree<H>(ch, nodes, first, 0);
}
// last levels (count <= 512): one block per tree, LDS
__global__ __launch_bounds__(256) void tree_top_kernel(Digest* nodes_all, u64 node_stride, u64 count) {
    __shared__ Digest lds[256];
    Digest* nodes = nodes_all + (u64)blockIdx.x * node_stride;
    const int tid = threadIdx.x;
    for (u64 c = count; c > 1; c >>= 1) {
        const u64 half = c >> 1;
        Digest d;
        if (tid < (int)half) {
            if (c == count) d = b3_merge(nodes[c + 2 * tid], nodes[c + 2 * tid + 1]);
            else d = b3_merge(lds[2 * tid], lds[2 * tid + 1]);
        }
        __syncthreads();
        if (tid < (int)half) {
            lds[tid] = d;
            nodes[half + tid] = d;
        }
        __syncthreads();
    }
}
void launch_tree_top(Digest* nodes, u64 node_stride, u64 count, int npoly, hipStream_t s) {
    while (count > 512) {
        int lg = 0;
        while ((1ULL << (lg + 1)) <= count) lg++;
        int h = 1;  // one coalesced merge per thread per level (multi-level variants gather 2^h
                    // digests per lane uncoalesced and measured slower)
        u64 outc = count >> h;
        dim3 g((unsigned)((outc + 255) / 256), npoly);
        if (h == 3) hipLaunchKernelGGL(tree_up_kernel<3>, g, dim3(256), 0, s, nodes, node_stride, count);
        else if (h == 2) hipLaunchKernelGGL(tree_up_kernel<2>, g, dim3(256), 0, s, nodes, node_stride, count);
        else hipLaunchKernelGGL(tree_up_kernel<1>, g, dim3(256), 0, s, nodes, node_stride, count);
        count = outc;
    }
    if (count > 1) {
        int threads = (int)(count / 2);
        threads = threads < 64 ? 64 : threads;
        hipLaunchKernelGGL(tree_top_kernel, dim3(npoly), dim3(threads), 0, s, nodes, node_stride, count);
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
__global__ __launch_bounds__(256) void fri_leaves_kernel(const u64* vals, u64 val_stride, int coset_major, int logn,
                                                         int logbeta, u64 rows, Digest* nodes_all, u64 node_stride) {
    const int proof = blockIdx.y;
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    const u64* base = vals + (u64)proof * val_stride;
    u64 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = layer_at(base, coset_major, logn, logbeta, i + (u64)k * rows);
    nodes_all[(u64)proof * node_stride + rows + i] = b3_hash_elems<8>(v);
}
void launch_fri_leaves(const u64* vals, u64 val_stride, bool coset_major, int logn, int logbeta, u64 rows,
                       Digest* nodes, u64 node_stride, int npoly, hipStream_t s) {
    dim3 g((unsigned)((rows + 255) / 256), npoly);
    hipLaunchKernelGGL(fri_leaves_kernel, g, dim3(256), 0, s, vals, val_stride, coset_major ? 1 : 0, logn, logbeta,
                       rows, nodes, node_stride);
    XFG_CHECK_LAUNCH();
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
__global__ __launch_bounds__(256) void constraint_eval_kernel(CeArgs a) {
    const u64 n = 1ULL << a.logn, nce = 2 * n;
    const int proof = blockIdx.y;
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // grid covers nce exactly
    const u64 par = g >> a.logn, m = g & (n - 1), i = 2 * m + par;
    const AirConst& A = a.air[proof];
    const u64* co = a.coeffs + (u64)proof * 15;
    const u64 beta = 1ULL << a.logbeta;
    const u64* lde = a.lde + (u64)proof * 7 * beta * n;
    const u64 t = par * (beta / 2), mn = (m + 1) & (n - 1);
    u64 cur[7];
#pragma unroll
    for (int c = 0; c < 7; c++) cur[c] = lde[(((u64)c << a.logbeta) + t) * n + m];
    const u64 nxt4 = lde[((4ULL << a.logbeta) + t) * n + mn];
    // XfgBurnMintAir::evaluate_transition (reference src/burn_mint_air.rs:335-378)
    const u64 std_burn = 8000000ULL, large_burn = 8000000000ULL;
    u64 r0 = gl_mul(gl_sub(cur[0], std_burn), gl_sub(cur[0], large_burn));
    u64 r1 = gl_sub(cur[1], cur[0]);
    u64 r2 = gl_sub(cur[2], A.pub[2] & 0xFFFFFFFFULL);
    u64 r3 = gl_sub(cur[3], A.pub[3] & 0xFFFFFFFFULL);
    u64 d = gl_sub(nxt4, cur[4]);
    u64 r4 = gl_mul(d, gl_sub(d, 1));
    u64 r5 = gl_sub(cur[5], A.nullifier);
    u64 r6 = gl_sub(cur[6], A.commitment);
    u64 tr = gl_mul(co[0], r0);
    tr = gl_add(tr, gl_mul(co[1], r1));
    tr = gl_add(tr, gl_mul(co[2], r2));
    tr = gl_add(tr, gl_mul(co[3], r3));
    tr = gl_add(tr, gl_mul(co[4], r4));
    tr = gl_add(tr, gl_mul(co[5], r5));
    tr = gl_add(tr, gl_mul(co[6], r6));
    // assertions (src/burn_mint_air.rs:380-395): step 0 on columns 0..6, step n-1 on column 4
    const u64 v0[7] = {A.pub[0], A.pub[1], A.pub[2], A.pub[3], 0, A.nullifier, A.commitment};
    u64 b0 = 0;
#pragma unroll
    for (int c = 0; c < 7; c++) b0 = gl_add(b0, gl_mul(co[7 + c], gl_sub(cur[c], v0[c])));
    u64 b1 = gl_mul(co[14], gl_sub(cur[4], 3));
    const u64 di = par * n + m;
    u64 val = gl_mul(tr, a.div[di]);
    val = gl_add(val, gl_mul(b0, a.div[nce + di]));
    val = gl_add(val, gl_mul(b1, a.div[2 * nce + di]));
    a.ce[(u64)proof * nce + i] = val;
}
void launch_constraint_eval(const u64* lde, const AirConst* air, const u64* coeffs, const u64* div, u64* ce, int logn,
                            int logbeta, int npoly, hipStream_t s) {
    CeArgs a;
    a.lde = lde; a.air = air; a.coeffs = coeffs; a.div = div; a.ce = ce; a.logn = logn; a.logbeta = logbeta;
    u64 nce = 2ULL << logn;
    int threads = nce < 256 ? (int)nce : 256;
    dim3 g((unsigned)(nce / threads), npoly);
    hipLaunchKernelGGL(constraint_eval_kernel, g, dim3(threads), 0, s, a);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ OOD
// partial sums of T_c(z), T_c(zg) (c < 7) and H(z); 8 consecutive coefficients per thread
__global__ __launch_bounds__(256) void ood_partial_kernel(const u64* coef, const u64* hcoef, const u64* zpts,
                                                          u64* partial, int logn) {
    __shared__ u64 red[15][256];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, tid = threadIdx.x;
    const u64 j0 = ((u64)blockIdx.x * blockDim.x + tid) * 8;
    const u64 z = zpts[2 * proof], zg = zpts[2 * proof + 1];
    u64 acc[15];
#pragma unroll
    for (int q = 0; q < 15; q++) acc[q] = 0;
    if (j0 < n) {
        u64 pz = gl_pow(z, j0), pzg = gl_pow(zg, j0);
        const u64* co = coef + (u64)proof * 7 * n;
        const u64* h = hcoef + (u64)proof * n;
        const int cnt = n - j0 < 8 ? (int)(n - j0) : 8;
        for (int r = 0; r < cnt; r++) {
            u64 j = j0 + r;
#pragma unroll
            for (int c = 0; c < 7; c++) {
                u64 v = co[(u64)c * n + j];
                acc[2 * c] = gl_add(acc[2 * c], gl_mul(v, pz));
                acc[2 * c + 1] = gl_add(acc[2 * c + 1], gl_mul(v, pzg));
            }
            acc[14] = gl_add(acc[14], gl_mul(h[j], pz));
            pz = gl_mul(pz, z);
            pzg = gl_mul(pzg, zg);
        }
    }
#pragma unroll
    for (int q = 0; q < 15; q++) red[q][tid] = acc[q];
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if (tid < off) {
#pragma unroll
            for (int q = 0; q < 15; q++) red[q][tid] = gl_add(red[q][tid], red[q][tid + off]);
        }
        __syncthreads();
    }
    for (int q = tid; q < 15; q += blockDim.x) partial[((u64)proof * gridDim.x + blockIdx.x) * 15 + q] = red[q][0];
}
__global__ void ood_final_kernel(const u64* partial, int nblk, u64* ood) {
    const int proof = blockIdx.x, q = threadIdx.x;
    if (q >= 15) return;
    u64 s = 0;
    for (int b = 0; b < nblk; b++) s = gl_add(s, partial[((u64)proof * nblk + b) * 15 + q]);
    ood[(u64)proof * 15 + q] = s;
}
void launch_ood(const u64* coef, const u64* hcoef, const u64* zpts, u64* partial, u64* ood, int logn, int npoly,
                hipStream_t s) {
    u64 n = 1ULL << logn;
    u64 nthreads = (n + 7) / 8;
    int threads = nthreads < 256 ? (int)nthreads : 256;
    int nblk = (int)((nthreads + threads - 1) / threads);
    hipLaunchKernelGGL(ood_partial_kernel, dim3(nblk, npoly), dim3(threads), 0, s, coef, hcoef, zpts, partial, logn);
    hipLaunchKernelGGL(ood_final_kernel, dim3(npoly), dim3(64), 0, s, partial, nblk, ood);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ DEEP
// P1_j = sum a_c T_c[j] + gamma H[j] - [j==0] c1 ; P2_j = sum a_c T_c[j] - [j==0] c2
// quotient of P/(x - b): q_k = sum_{j>k} P_j b^(j-k-1) = b^-(k+1) * sum_{j>k} P_j b^j
// s_j = P_j b^j (two streams) -> exclusive suffix sums -> d_k = z^-(k+1) E1_k + zg^-(k+1) E2_k
#define DEEP_PER_THREAD 8
__device__ __forceinline__ void deep_terms(const u64* co, const u64* h, const DeepParams& P, u64 n, u64 j, u64& p1,
                                           u64& p2) {
    u64 s = 0;
#pragma unroll
    for (int c = 0; c < 7; c++) s = gl_add(s, gl_mul(P.a[c], co[(u64)c * n + j]));
    p1 = gl_add(s, gl_mul(P.gamma, h[j]));
    p2 = s;
    if (j == 0) {
        p1 = gl_sub(p1, P.c1);
        p2 = gl_sub(p2, P.c2);
    }
}
__global__ __launch_bounds__(256) void deep_blocksum_kernel(const u64* coef, const u64* hcoef, const DeepParams* dp,
                                                            u64* bsum, int logn) {
    __shared__ u64 r1[256], r2[256];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, tid = threadIdx.x;
    const DeepParams P = dp[proof];
    const u64* co = coef + (u64)proof * 7 * n;
    const u64* h = hcoef + (u64)proof * n;
    const u64 j0 = ((u64)blockIdx.x * blockDim.x + tid) * DEEP_PER_THREAD;
    u64 s1 = 0, s2 = 0;
    if (j0 < n) {
        u64 pz = gl_pow(P.z, j0), pzg = gl_pow(P.zg, j0);
        for (int r = 0; r < DEEP_PER_THREAD && j0 + r < n; r++) {
            u64 p1, p2;
            deep_terms(co, h, P, n, j0 + r, p1, p2);
            s1 = gl_add(s1, gl_mul(p1, pz));
            s2 = gl_add(s2, gl_mul(p2, pzg));
            pz = gl_mul(pz, P.z);
            pzg = gl_mul(pzg, P.zg);
        }
    }
    r1[tid] = s1;
    r2[tid] = s2;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if (tid < off) {
            r1[tid] = gl_add(r1[tid], r1[tid + off]);
            r2[tid] = gl_add(r2[tid], r2[tid + off]);
        }
        __syncthreads();
    }
    if (tid == 0) {
        bsum[((u64)proof * gridDim.x + blockIdx.x) * 2] = r1[0];
        bsum[((u64)proof * gridDim.x + blockIdx.x) * 2 + 1] = r2[0];
    }
}
// exclusive suffix sums over blocks (serial per proof; nblk is small)
__global__ void deep_carry_kernel(const u64* bsum, u64* carry, int nblk) {
    const int proof = blockIdx.x, q = threadIdx.x;
    if (q >= 2) return;
    u64 s = 0;
    for (int b = nblk - 1; b >= 0; b--) {
        carry[((u64)proof * nblk + b) * 2 + q] = s;
        s = gl_add(s, bsum[((u64)proof * nblk + b) * 2 + q]);
    }
}
__global__ __launch_bounds__(256) void deep_final_kernel(const u64* coef, const u64* hcoef, const DeepParams* dp,
                                                         const u64* carry, u64* deep, int logn) {
    __shared__ u64 e1[256], e2[256];
    const u64 n = 1ULL << logn;
    const int proof = blockIdx.y, tid = threadIdx.x, T = blockDim.x;
    const DeepParams P = dp[proof];
    const u64* co = coef + (u64)proof * 7 * n;
    const u64* h = hcoef + (u64)proof * n;
    const u64 j0 = ((u64)blockIdx.x * T + tid) * DEEP_PER_THREAD;
    u64 s1[DEEP_PER_THREAD], s2[DEEP_PER_THREAD];
    u64 t1 = 0, t2 = 0;
    {
        u64 pz = j0 < n ? gl_pow(P.z, j0) : 0, pzg = j0 < n ? gl_pow(P.zg, j0) : 0;
#pragma unroll
        for (int r = 0; r < DEEP_PER_THREAD; r++) {
            s1[r] = s2[r] = 0;
            if (j0 + r < n) {
                u64 p1, p2;
                deep_terms(co, h, P, n, j0 + r, p1, p2);
                s1[r] = gl_mul(p1, pz);
                s2[r] = gl_mul(p2, pzg);
                pz = gl_mul(pz, P.z);
                pzg = gl_mul(pzg, P.zg);
            }
            t1 = gl_add(t1, s1[r]);
            t2 = gl_add(t2, s2[r]);
        }
    }
    // inclusive suffix scan of per-thread totals
    e1[tid] = t1;
    e2[tid] = t2;
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {
        u64 a1 = e1[tid], a2 = e2[tid];
        if (tid + off < T) {
            a1 = gl_add(a1, e1[tid + off]);
            a2 = gl_add(a2, e2[tid + off]);
        }
        __syncthreads();
        e1[tid] = a1;
        e2[tid] = a2;
        __syncthreads();
    }
    // exclusive suffix (everything after this thread's chunk) + blocks after this one
    u64 c1 = carry[((u64)proof * gridDim.x + blockIdx.x) * 2];
    u64 c2 = carry[((u64)proof * gridDim.x + blockIdx.x) * 2 + 1];
    u64 x1 = gl_add(c1, tid + 1 < T ? e1[tid + 1] : 0);
    u64 x2 = gl_add(c2, tid + 1 < T ? e2[tid + 1] : 0);
    if (j0 >= n) return;
    // walk the chunk backwards: E_k = sum_{j>k} s_j
    const int cnt = n - j0 < DEEP_PER_THREAD ? (int)(n - j0) : DEEP_PER_THREAD;
    u64 last = j0 + cnt - 1;
    u64 iz = gl_pow(P.zinv, last + 1), izg = gl_pow(P.zginv, last + 1);
    u64* out = deep + (u64)proof * n;
    for (int r = cnt - 1; r >= 0; r--) {
        out[j0 + r] = gl_add(gl_mul(iz, x1), gl_mul(izg, x2));
        x1 = gl_add(x1, s1[r]);
        x2 = gl_add(x2, s2[r]);
        iz = gl_mul(iz, P.z);
        izg = gl_mul(izg, P.zg);
    }
}
void launch_deep(const u64* coef, const u64* hcoef, const DeepParams* dp, u64* bsum, u64* carry, u64* deep, int logn,
                 int npoly, hipStream_t s) {
    u64 n = 1ULL << logn;
    u64 nthreads = (n + DEEP_PER_THREAD - 1) / DEEP_PER_THREAD;
    int threads = nthreads < 256 ? (int)nthreads : 256;
    int nblk = (int)((nthreads + threads - 1) / threads);
    hipLaunchKernelGGL(deep_blocksum_kernel, dim3(nblk, npoly), dim3(threads), 0, s, coef, hcoef, dp, bsum, logn);
    hipLaunchKernelGGL(deep_carry_kernel, dim3(npoly), dim3(64), 0, s, bsum, carry, nblk);
    hipLaunchKernelGGL(deep_final_kernel, dim3(nblk, npoly), dim3(threads), 0, s, coef, hcoef, dp, carry, deep, logn);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ FRI fold
// apply_drp for folding factor 8 with Winterfell's constant domain offset 7 on every layer:
// row i = {v_k at 7 w_D^i zeta^k}; c = iDFT_8(v)/8 ; result = sum_j c_j (alpha / (7 w_D^i))^j
struct FoldArgs {
    const u64* vals;
    u64 val_stride;
    int coset_major, logn, logbeta;
    u64 rows;
    int logD;
    const u64* alpha7;
    u64* out;
    u64 out_stride;
    u64 winv8[4];  // w_8^-k, k < 4
    u64 inv8;
    Tables T;
};
__global__ __launch_bounds__(256) void fri_fold_kernel(FoldArgs a) {
    const int proof = blockIdx.y;
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.rows) return;
    const u64* base = a.vals + (u64)proof * a.val_stride;
    u64 v[8];
    // bit-reversed load for an in-register radix-2 DIT inverse DFT of size 8
    const int br[8] = {0, 4, 2, 6, 1, 5, 3, 7};
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = layer_at(base, a.coset_major, a.logn, a.logbeta, i + (u64)br[k] * a.rows);
#pragma unroll
    for (int s = 0; s < 3; s++) {
        const int h = 1 << s;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            int pos = b & (h - 1), i0 = ((b >> s) << (s + 1)) + pos;
            u64 w = a.winv8[pos << (2 - s)];
            u64 u = v[i0], t = gl_mul(v[i0 + h], w);
            v[i0] = gl_add(u, t);
            v[i0 + h] = gl_sub(u, t);
        }
    }
    // y = alpha * 7^-1 * w_D^-i ; Horner
    u64 y = gl_mul(a.alpha7[proof], tw_ipow(a.T, a.logD, i));
    u64 r = v[7];
#pragma unroll
    for (int j = 6; j >= 0; j--) r = gl_add(gl_mul(r, y), v[j]);
    a.out[(u64)proof * a.out_stride + i] = gl_mul(r, a.inv8);
}
void launch_fri_fold(const u64* vals, u64 val_stride, bool coset_major, int logn, int logbeta, u64 rows, int logD,
                     const u64* alpha7, u64* out, u64 out_stride, const Tables& T, int npoly, hipStream_t s) {
    FoldArgs a;
    a.vals = vals; a.val_stride = val_stride; a.coset_major = coset_major ? 1 : 0; a.logn = logn;
    a.logbeta = logbeta; a.rows = rows; a.logD = logD; a.alpha7 = alpha7; a.out = out; a.out_stride = out_stride;
    a.T = T;
    u64 w8inv = gl_inv(gl_root(3));
    for (int k = 0; k < 4; k++) a.winv8[k] = gl_pow(w8inv, k);
    a.inv8 = gl_inv(8);
    int threads = rows < 256 ? (int)rows : 256;
    dim3 g((unsigned)((rows + threads - 1) / threads), npoly);
    hipLaunchKernelGGL(fri_fold_kernel, g, dim3(threads), 0, s, a);
    XFG_CHECK_LAUNCH();
}

// ============================================================================ gathers
__global__ void gather_u64_kernel(const u64* src, const u64* idx, u64* dst, u64 count) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = src[idx[i]];
}
__global__ void gather_digest_kernel(const Digest* src, const u64* idx, Digest* dst, u64 count) {
    u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = src[idx[i]];
}
void launch_gather_u64(const u64* src, const u64* idx, u64* dst, u64 count, hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(gather_u64_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, src, idx, dst, count);
}
void launch_gather_digest(const Digest* src, const u64* idx, Digest* dst, u64 count, hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(gather_digest_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, src, idx, dst,
                       count);
}

}  // namespace xfg
