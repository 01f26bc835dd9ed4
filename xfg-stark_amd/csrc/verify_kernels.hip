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

__global__ void vgather_kernel(const uint8_t* blob, const VGather* g, u64 n, Digest* dig) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = blob + g[i].src;
    Digest d;
#pragma unroll
    for (int w = 0; w < 8; w++)
        d.w[w] = (uint32_t)p[4 * w] | ((uint32_t)p[4 * w + 1] << 8) | ((uint32_t)p[4 * w + 2] << 16) |
                 ((uint32_t)p[4 * w + 3] << 24);
    dig[g[i].dst] = d;
}

template <int K>
__device__ __forceinline__ Digest hash_words(const uint8_t* p) {
    u64 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = ld_u64(p + 8 * k);
    return b3_hash_elems<K>(v);
}
__global__ void vleaf_kernel(const uint8_t* blob, const VLeaf* lv, u64 n, Digest* dig) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const VLeaf L = lv[i];
    const uint8_t* p = blob + L.src;
    Digest d;
    switch (L.words) {  // trace row 7, constraint value 1 / 2, FRI row 8 / 16
        case 1: d = hash_words<1>(p); break;
        case 2: d = hash_words<2>(p); break;
        case 7: d = hash_words<7>(p); break;
        case 8: d = hash_words<8>(p); break;
        default: d = hash_words<16>(p); break;
    }
    dig[L.dst] = d;
}
__global__ void vmerge_kernel(const uint32_t* t, u64 n, Digest* dig) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dig[t[3 * i]] = b3_merge(dig[t[3 * i + 1]], dig[t[3 * i + 2]]);
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

void launch_verify(const uint8_t* blob, const VGather* g, u64 ng, const VLeaf* lv, u64 nleaf,
                   const uint32_t* rounds, const u64* round_off, int nrounds, const VFieldProof* fp,
                   const VFieldQuery* fq, u64 nq, Digest* dig, uint32_t* flags, hipStream_t s) {
    if (ng) hipLaunchKernelGGL(vgather_kernel, dim3(blocks_for(ng, 256)), dim3(256), 0, s, blob, g, ng, dig);
    if (nleaf) hipLaunchKernelGGL(vleaf_kernel, dim3(blocks_for(nleaf, 256)), dim3(256), 0, s, blob, lv, nleaf, dig);
    for (int r = 0; r < nrounds; r++) {
        const u64 cnt = (round_off[r + 1] - round_off[r]) / 3;
        if (cnt)
            hipLaunchKernelGGL(vmerge_kernel, dim3(blocks_for(cnt, 256)), dim3(256), 0, s, rounds + round_off[r], cnt,
                               dig);
    }
    if (nq) hipLaunchKernelGGL(vfield_kernel, dim3(blocks_for(nq, 64)), dim3(64), 0, s, blob, fp, fq, nq, flags);
    (void)hipGetLastError();
}

}  // namespace xfg
