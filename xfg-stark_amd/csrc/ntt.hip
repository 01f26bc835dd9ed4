// Four-step Goldilocks NTT for CDNA4 (gfx950): coset LDE and (coset) interpolation.
//
// Replaces winter-math fft::interpolate_poly / evaluate_poly_with_offset as used by Winterfell's
// DefaultTraceLde, CompositionPoly and DeepCompositionPoly (the LDE behind
// src/burn_mint_air.rs:504-514 `new_trace_lde`).
//
// n = R * C. Pass A: size-R DFTs down the columns of the [R][C] view, pass B: size-C DFTs
// along the rows. Each pass is a chain of Stockham autosort steps with radix-16 butterflies in
// registers (16 elements per thread, 256 threads, 4096-element tiles):
//   * the first step of a pass loads straight from HBM (coalesced: 16 lanes cover 128 B),
//   * the middle steps go through one padded LDS tile,
//   * the last step stores straight to HBM, applying the four-step / coset twiddles as running
//     products (2 table reads per thread, no per-element twiddle-table gathers).
// Twiddles inside a radix-16 butterfly are 16th roots of unity = powers of two in Goldilocks
// (w_16 = 2^156, w_8 = 2^120, w_4 = 2^48, w_2 = 2^96 = -1): shifts + one reduction.
//
// Forward LDE output is coset-major: out[p][t][m] = P(7 * w_N^(t + beta*m)), N = beta * n.
// The coset shift (7 w_N^t)^j, j = C j1 + j2, is split into a pre-factor 7^(C j1) w_(beta R)^(t j1)
// (LDS table per coset) and a post-factor 7^j2 w_N^(j2 t) folded into the four-step twiddle.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include "kernels.hpp"
#include "field_dft.hpp"

namespace xfg {

// Raw buffer access for the passes' strided global loads / stores: the per-lane part of an address
// is a 32-bit VGPR offset computed once per group, the part that varies with the butterfly output
// r (r * stride rows) is wave-uniform and goes in the SGPR offset -- no 64-bit address arithmetic
// on the VALU per element. Bases are per (poly, coset) planes, so offsets stay below 2^32 bytes.
typedef u32 u32x2 __attribute__((__vector_size__(8)));
// p must be wave-uniform; it is read from the first lane so that the descriptor is built in SGPRs
// (a descriptor the compiler cannot prove uniform gets a readfirstlane/compare loop around every
// access)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const u64* p) {
    const u64 a = (u64)p;
    const u64 u = (u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)a) |
                  ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(a >> 32)) << 32);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ u64 buf_ld(__amdgpu_buffer_rsrc_t r, u32 voff, u32 soff) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
    return (u64)v[0] | ((u64)v[1] << 32);
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, u32 voff, u32 soff, u64 x) {
    const u32x2 v = {(u32)x, (u32)(x >> 32)};
    __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)voff, (int)soff, 0);
}

// 16-byte stores of column pairs. A pass's last step leaves each lane the outputs of one column (pass
// A) or row (pass B) at rows / positions base + r * stride, and lanes 2i, 2i + 1 hold the two
// neighbouring words of every such output line. One dword pair swapped between them (DPP quad_perm
// [1, 0, 3, 2], folded into the selects) lets the even lane store both words of the even outputs and
// the odd lane both words of the odd ones: half as many store instructions, 16 B per lane. (A wave
// ending a tile with 32 8-byte stores per lane is store-issue-bound: MI355X_MICROARCH.md, "store
// tail".) Full tiles only: both lanes of a pair must hold a group.
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64 swap_lane_pair(u64 x) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(u32)x, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(u32)(x >> 32), 0xB1, 0xF, 0xF, false);
    return (u64)(u32)lo | ((u64)(u32)hi << 32);
}
// The same pairing through a buffer resource: output r of the pair's even word sits at byte offset
// vo + r * step (vo per lane, step wave-uniform), so the part that varies with r rides in the SGPR
// offset and no 64-bit address is computed per store (the odd lane stores output r + 1: its extra
// `step` goes into its VGPR offset once)
typedef u32 u32x4 __attribute__((__vector_size__(16)));
template <int RR>
__device__ __forceinline__ void store_pairs_buf(const u64* v, __amdgpu_buffer_rsrc_t rs, u32 vo, u32 step) {
    const bool odd = threadIdx.x & 1;
    const u32 vl = vo + (odd ? step : 0u);
#pragma unroll
    for (int r = 0; r < RR; r += 2) {
        const u64 g0 = swap_lane_pair(v[r]), g1 = swap_lane_pair(v[r + 1]);
        const u64 lo = odd ? g1 : v[r], hi = odd ? v[r + 1] : g0;
        const u32x4 d = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)vl, (int)((u32)r * step), 0);
    }
}
// at(r): address of output r of the pair's EVEN word (16-byte aligned)
template <int RR, class AT>
__device__ __forceinline__ void store_pairs(const u64* v, AT at) {
    const bool odd = threadIdx.x & 1;
#pragma unroll
    for (int r = 0; r < RR; r += 2) {
        const u64 g0 = swap_lane_pair(v[r]), g1 = swap_lane_pair(v[r + 1]);
        const u64x2 d = {odd ? g1 : v[r], odd ? v[r + 1] : g0};
        *reinterpret_cast<u64x2*>(at(odd ? r + 1 : r)) = d;
    }
}

// LDS tile: row `seq` of length S at seq * PITCH; element i at i + (i >> P), one pad word per 2^P
// elements, P = log2 elements per thread (4 or 5). The pad word makes the stride-2^P stores of a
// full-radix first step (lanes along a row, 2^P contiguous outputs each) conflict-free: 16 lanes
// land on 16 different 8-byte bank pairs. The pitch does the same for lanes walking across rows:
// a 16-lane group spans 2^L rows and 16 / 2^L consecutive elements, so the pitch must be an odd
// multiple of 16 / 2^L mod 16 (radix 16: odd; radix 32 with 8-row tiles, pass B at n = 2^20: 2 mod
// 4 -- the odd pitch there cost 2-way conflicts on every last-step read, and the pad per 16 on
// every first-step write, 14.8 M conflict cycles per configs[4] trace LDE).
// L = log2 of the tile's row count (the kernel's maximum; a smaller tile only uses fewer rows).
__host__ __device__ constexpr int row_pitch(int S, int P = 4, int L = 4) {
    return P == 4 ? S + S / 16 + 1 : S + (S >> P) + ((L >= 4 || L <= 0) ? 1 : (16 >> L));
}
// Pitch of a 32-bit exchange tile (pass_dft_split). Its writes and ds_read_b32 / ds_read2_b32 reads
// bank on (a / 4) mod 32 per 32-lane half, where a row-fast half-wave spans 2^L rows of the tile and
// 32 / 2^L consecutive groups, so a row pitch of 32 / 2^L (mod 32) spreads the rows over distinct bank
// groups. Radix 32 (P = 5): S + S / 32 + 32 / 2^L (the 64-bit pitch, 2 mod 32 at 8 rows, was 2-way
// conflicted on pass A's first-step writes and both passes' second-step reads: 22 M conflict cycles
// per configs[4] trace LDE). Radix 16 keeps row_pitch.
__host__ __device__ constexpr int split_pitch(int S, int P, int L) {
    return P == 5 ? S + (S >> 5) + ((32 >> L) & 31) : row_pitch(S, P, L);
}
template <int P>
__device__ __forceinline__ int phys(int i) { return i + (i >> P); }
// phys(j + o) for an offset o that is a compile-time constant after unrolling: a multiple of 2^P
// splits off as a constant (the LDS instruction's immediate offset), so the per-lane index
// phys(j) is computed once per group instead of once per element
template <int P>
__device__ __forceinline__ int phys2(int j, int o) {
    return (o & ((1 << P) - 1)) == 0 ? phys<P>(j) + o + (o >> P) : phys<P>(j + o);
}

__device__ __forceinline__ u64 tw_get(const Tables& T, int k, u64 e, bool inv) {
    const u64 M = 1ULL << T.LM;
    u64 idx = (e << (T.LM - k)) & (M - 1);
    if (inv) idx = (M - idx) & (M - 1);
    return T.tw[idx];
}

// ---------------------------------------------------------------- one Stockham step
// Radix 2^LOGR step of a size-2^LOGS DFT on 2^lognseq sequences, 2^LOGE elements per thread
// (2^(LOGE - LOGR) groups). Group g of the step is
// (seq, j); SEQ_FAST maps consecutive lanes to consecutive sequences, otherwise to consecutive j.
// ld(seq, j, o) reads logical element i = j + o of a sequence (o = r * G, uniform across the
// wave); st(seq, base, stride, v) receives the R
// outputs of a group, which belong at logical positions base + r * stride.
// IN_PLACE: every load of the step completes (barrier) before any store.
// pf(q, seq, base, stride) runs before the group's loads (prefetch of what st will need).
// TW2D: the twiddle of element r of a group with k = j % Ns is ltw[r * Ns + k] (a per-step [r][k]
// table, ntt_pass_a_cos2) instead of w^(r k step) = ltw[r * k * step]
template <int LOGS, int LOGR, int LOGE, bool INV, bool SEQ_FAST, bool IN_PLACE, int NT, class LD, class ST, class PF,
          bool TW2D = false, bool CANON_OUT = false>
__device__ __forceinline__ void stockham(int lognseq, int Ns, const u64* ltw, LD ld, ST st, PF pf) {
    constexpr int S = 1 << LOGS, R = 1 << LOGR, G = S / R, PER = (1 << LOGE) / R;
    const int nseq = 1 << lognseq;
    const int groups = nseq * G;
    u64 v[PER][R];
    int gs[PER], gj[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        // lanes past the last group (partial tiles only) recompute the last group and drop the
        // result: no divergent branch, and no zero-initialised registers for the untaken path
        const int g0 = threadIdx.x + NT * q, g = g0 < groups ? g0 : groups - 1;
        const int seq = SEQ_FAST ? (g & (nseq - 1)) : (g / G);
        const int j = SEQ_FAST ? (g >> lognseq) : (g % G);
        pf(q, seq, (j / Ns) * Ns * R + (j % Ns), Ns);
#pragma unroll
        for (int r = 0; r < R; r++) v[q][r] = ld(seq, j, r * G);
        if (Ns > 1) {
            const int k = j % Ns, step = S / (Ns * R);
            // in pairs (gl_mul2: each product's carry wait states filled by the other's instructions)
#pragma unroll
            for (int r = 1; r + 1 < R; r += 2)
                gl_mul2(v[q][r], TW2D ? ltw[r * Ns + k] : ltw[r * k * step], v[q][r + 1],
                        TW2D ? ltw[(r + 1) * Ns + k] : ltw[(r + 1) * k * step]);
            v[q][R - 1] = gl_mul(v[q][R - 1], TW2D ? ltw[(R - 1) * Ns + k] : ltw[(R - 1) * k * step]);
        }
        dft_reg<LOGR, INV, CANON_OUT>(v[q]);
        gs[q] = g0 < groups ? seq : -1;
        gj[q] = j;
    }
    if (IN_PLACE) __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        if (gs[q] >= 0) {
            const int j = gj[q];
            st(q, gs[q], (j / Ns) * Ns * R + (j % Ns), Ns, v[q]);
        }
    }
}

// steps of a size-2^LOGS DFT with 2^LOGE elements per thread: the remainder radix first, then
// radix 2^LOGE (16, or 32 where that saves a general-twiddle step: a size-1024 DFT is 32 x 32
// -- one twiddle multiply per element -- instead of 4 x 16 x 16 -- two; the radix-32 butterfly
// twiddles are still shifts, w_32 = 2^78). (Remainder last would save general twiddle multiplies
// -- radix 2 last multiplies 1/2 of the elements where radix 2 first makes the next radix-16 step
// multiply 15/16 -- but its narrow final step stores measured 25 % slower at 2^20: 2.14 vs
// 1.72 ms per configs[4] trace LDE, same box.)
template <int LOGS, int LOGE = 4>
struct Plan {
    static constexpr int REM = LOGS % LOGE;
    static constexpr int NSTEP = LOGS / LOGE + (REM ? 1 : 0);
    static constexpr int FIRST_LOGR = REM ? REM : LOGE;
    // radix of the step that produces the final outputs
    static constexpr int LAST_LOGR = NSTEP == 1 ? FIRST_LOGR : LOGE;
    static constexpr int LAST_R = 1 << LAST_LOGR;
};

// Whole DFT of every sequence: the first step loads with ldg (global), middle steps run in the
// LDS tile, the last step stores with stg (global). A one-step DFT goes global -> global.
// stg(q, seq, base, stride, v) stores group q's outputs; pf as in stockham, for the last step
constexpr int NT_LOG2(int nt) { return nt <= 1 ? 0 : 1 + NT_LOG2(nt / 2); }
template <int LOGS, int LOGE, bool INV, bool FIRST_SEQ_FAST, int NT, class LDG, class STG, class PF, bool TW2D_LAST = false>
__device__ __forceinline__ void pass_dft(u64* tile, int lognseq, const u64* ltw, LDG ldg, STG stg, PF pf) {
    using PL = Plan<LOGS, LOGE>;
    constexpr int L = NT_LOG2(NT) + LOGE - LOGS;
    constexpr int PITCH = row_pitch(1 << LOGS, LOGE, L), E = 1 << LOGE;
    auto nopf = [](int, int, int, int) {};
    if constexpr (PL::NSTEP == 1) {
        stockham<LOGS, PL::FIRST_LOGR, LOGE, INV, FIRST_SEQ_FAST, false, NT>(lognseq, 1, ltw, ldg, stg, pf);
    } else {
        stockham<LOGS, PL::FIRST_LOGR, LOGE, INV, FIRST_SEQ_FAST, false, NT>(
            lognseq, 1, ltw, ldg, [&](int, int seq, int base, int stride, u64* v) {
                u64* row = tile + seq * PITCH;
#pragma unroll
                for (int r = 0; r < (1 << PL::FIRST_LOGR); r++) {
                    // full-radix first step: base = R j, stride 1 -> the R outputs are contiguous
                    // (a multiple of 16 elements: the pad words fall at fixed offsets)
                    if constexpr (PL::FIRST_LOGR >= 4) row[phys<LOGE>(base) + r + (r >> LOGE)] = v[r];
                    else row[phys<LOGE>(base + r * stride)] = v[r];
                }
            },
            nopf);
        __syncthreads();
        int Ns = 1 << PL::FIRST_LOGR;
        auto ldl = [&](int seq, int j, int o) { return tile[seq * PITCH + phys2<LOGE>(j, o)]; };
#pragma unroll
        for (int st = 1; st < PL::NSTEP - 1; st++) {
            stockham<LOGS, LOGE, LOGE, INV, true, true, NT>(
                lognseq, Ns, ltw, [&](int seq, int j, int o) { return tile[seq * PITCH + phys2<LOGE>(j, o)]; },
                [&](int, int seq, int base, int stride, u64* v) {
                    u64* row = tile + seq * PITCH;
#pragma unroll
                    for (int r = 0; r < E; r++) row[phys2<LOGE>(base, r * stride)] = v[r];
                },
                nopf);
            __syncthreads();
            Ns <<= LOGE;
        }
        stockham<LOGS, PL::LAST_LOGR, LOGE, INV, true, false, NT, decltype(ldl), STG, PF, TW2D_LAST>(lognseq, Ns, ltw,
                                                                                                ldl, stg, pf);
        __syncthreads();
    }
}

// pass_dft for two full-radix steps (one group per thread, full tiles) with the exchange between the
// steps in 32-bit halves: the low words go through the LDS tile, then the high words through the
// same tile, so the tile is half the size of a 64-bit one and twice as many blocks fit a CU. Costs
// twice the LDS instructions and two more barriers per tile.
template <int LOGS, int LOGE, bool INV, bool FIRST_SEQ_FAST, int NT, class LDG, class STG, class PF, bool TW2D_LAST = false,
          bool CANON_OUT = false>
__device__ __forceinline__ void pass_dft_split(u32* tile, int lognseq, const u64* ltw, LDG ldg, STG stg, PF pf) {
    using PL = Plan<LOGS, LOGE>;
    static_assert(PL::NSTEP == 2 && PL::FIRST_LOGR == LOGE, "two full-radix steps");
    constexpr int L = NT_LOG2(NT) + LOGE - LOGS;
    constexpr int PITCH = split_pitch(1 << LOGS, LOGE, L), E = 1 << LOGE, G = (1 << LOGS) / E;
    auto nopf = [](int, int, int, int) {};
    u32 hi[E];
    int sseq = 0, sbase = 0;
    stockham<LOGS, LOGE, LOGE, INV, FIRST_SEQ_FAST, false, NT>(
        lognseq, 1, ltw, ldg,
        [&](int, int seq, int base, int, u64* v) {
            u32* row = tile + seq * PITCH + phys<LOGE>(base);
#pragma unroll
            for (int r = 0; r < E; r++) {
                row[r + (r >> LOGE)] = (u32)v[r];
                hi[r] = (u32)(v[r] >> 32);
            }
            sseq = seq;
            sbase = base;
        },
        nopf);
    __syncthreads();
    // this thread's group of the second step (stockham, SEQ_FAST, q = 0)
    const int g = threadIdx.x, seq = g & ((1 << lognseq) - 1), j = g >> lognseq;
    u32 lo[E];
#pragma unroll
    for (int r = 0; r < E; r++) lo[r] = tile[seq * PITCH + phys2<LOGE>(j, r * G)];
    __syncthreads();
    {
        u32* row = tile + sseq * PITCH + phys<LOGE>(sbase);
#pragma unroll
        for (int r = 0; r < E; r++) row[r + (r >> LOGE)] = hi[r];
    }
    __syncthreads();
    auto ldl = [&](int sq, int jj, int o) { return (u64)lo[o / G] | ((u64)tile[sq * PITCH + phys2<LOGE>(jj, o)] << 32); };
    stockham<LOGS, LOGE, LOGE, INV, true, false, NT, decltype(ldl), STG, PF, TW2D_LAST, CANON_OUT>(lognseq, E, ltw, ldl, stg,
                                                                                                 pf);
    __syncthreads();
}

__host__ __device__ u64 fourstep_main(int logn, int logbeta);
struct NttArgs {
    const u64* in;
    u64* y;
    u64* out;
    u64 in_stride, out_stride;
    int logn, logR, logC;
    int logbeta;  // forward: 2^logbeta cosets
    int off7;     // inverse: scale coefficient k by 7^-k
    u64 scale;    // inverse: n^-1
    u64 keep;     // inverse: coefficients written
    const u64* t4;  // four-step twiddle table (FourStep) or nullptr
    const u64* pt;  // pass tables: w_R^(+-i) [R], w_C^(+-i) [C], forward coset pre-factors [beta][R]; or nullptr
    int xcd;        // 1 / 2: XCD-contiguous block order of pass A / B (xcd_block); 4: pass A cosets
                    // of a tile consecutive (xcd_block_coset)
    int tq_b;       // forward: pass B applies the four-step twiddles as it loads (ntt_pass_a_cos)
    int preg;       // forward pass A: coset pre-factors read from the pass tables in L2, not LDS
    Tables T;
};

// Workgroups are dealt round-robin over the 8 XCDs, each with its own L2. When a pass writes less
// than a 128 B line per tile row, the neighbouring tiles that fill the rest of each line must run
// on the same XCD at about the same time or every line reaches HBM in pieces: renumber so that
// XCD x executes the x-th contiguous eighth of the (tile, poly) blocks in order.
__device__ __forceinline__ void xcd_block(bool on, int& bx, int& by) {
    if (!on) {
        bx = blockIdx.x;
        by = blockIdx.y;
        return;
    }
    const int total = gridDim.x * gridDim.y, L = blockIdx.x + gridDim.x * blockIdx.y;
    const int per = total >> 3, rem = total & 7, x = L & 7, slot = L >> 3;
    const int l = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + slot;
    bx = l % gridDim.x;
    by = l / gridDim.x;
}

// The same XCD-contiguous renumbering with the cosets of a (poly, column tile) consecutive: the
// beta blocks that read one coefficient tile then run side by side on one XCD, so the tile comes
// from HBM once and from that XCD's L2 beta - 1 times (forward pass A without the all-coset kernel:
// configs[4]'s R = 1024); the two 64 B halves of an intermediate line (tiles 2i, 2i + 1 of a coset)
// are written 2^logbeta blocks apart on the same XCD.
__device__ __forceinline__ void xcd_block_coset(int logbeta, int& bx, int& by) {
    const int total = gridDim.x * gridDim.y, L = blockIdx.x + gridDim.x * blockIdx.y;
    const int per = total >> 3, rem = total & 7, x = L & 7, slot = L >> 3;
    const int l = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + slot;
    const int t = l & ((1 << logbeta) - 1), rest = l >> logbeta;
    bx = rest % gridDim.x;
    by = ((rest / gridDim.x) << logbeta) + t;
}

// ---------------------------------------------------------------- pass A: column DFTs (size R)
// forward, coset t: x[j1] = c[C j1 + j2] * 7^(C j1) w_(beta R)^(t j1)
//   y[t][k1][j2] = X[k1] * 7^j2 * w_N^(j2 (t + beta k1))
// inverse: y[k1][j2] = X[k1] * w_n^-(j2 k1)
// LOGT = log2 threads, LOGE = log2 elements per thread: 2^(LOGT + LOGE)-element tiles, e.g.
// 256 x 16 (several blocks per CU), 1024 x 16 or 512 x 32 (16384 elements in up to 155 KiB of
// LDS, one block per CU: 16 columns per tile even at R = 1024)
template <int LOGR, bool INV, int LOGT, int LOGE>
__global__ __launch_bounds__(1 << LOGT, (1 << (10 - LOGT)) >> (LOGE - 4)) void ntt_pass_a(NttArgs a) {
    constexpr int R = 1 << LOGR, PITCH = row_pitch(R, LOGE, LOGT + LOGE - LOGR), RR = Plan<LOGR, LOGE>::LAST_R,
                  NT = 1 << LOGT;
    extern __shared__ u64 lds[];
    const int logTC = (a.logC < LOGT + LOGE - LOGR) ? a.logC : LOGT + LOGE - LOGR;
    const int TC = 1 << logTC;
    u64* tile = lds;
    u64* ltw = lds + TC * PITCH;
    u64* pre = ltw + R;  // forward: 7^(C j1) w_(beta R)^(t j1) for this block's coset
    // one block per (column tile, poly, coset); y is [poly][coset][R][C]
    int bx, by;
    if (!INV && (a.xcd & 4)) xcd_block_coset(a.logbeta, bx, by);
    else xcd_block(a.xcd & 1, bx, by);
    const int pt = by, col0 = bx * TC;
    const int poly = INV ? pt : (pt >> a.logbeta), t = INV ? 0 : (pt & ((1 << a.logbeta) - 1));
    const u64 n = 1ULL << a.logn;
    const int logN = a.logn + a.logbeta;
    const u64 maskN = (1ULL << logN) - 1;
    if (a.pt) {
        // contiguous per-size tables (behind the four-step table, or standalone): coalesced loads
        for (int i = threadIdx.x; i < R; i += NT) {
            ltw[i] = a.pt[i];
            if (!INV && !a.preg) pre[i] = a.pt[R + (1 << a.logC) + t * R + i];
        }
    } else {
        for (int i = threadIdx.x; i < R; i += NT) {
            ltw[i] = tw_get(a.T, LOGR, i, INV);
            if (!INV)
                pre[i] = gl_mul(a.T.pow7[(u64)i << a.logC],
                                tw_get(a.T, LOGR + a.logbeta, ((u64)t * i) & ((1ULL << (LOGR + a.logbeta)) - 1), false));
        }
    }
    __syncthreads();
    const u64* in = a.in + (u64)poly * a.in_stride;
    u64* y = a.y + (u64)pt * n;
    const auto rin = buf_rsrc(in + col0), ry = buf_rsrc(y + col0);
    const u64* preg = (!INV && a.preg) ? a.pt + R + (1 << a.logC) + (u64)t * R : nullptr;
    auto ldg = [&](int seq, int j, int o) -> u64 {
        const u64 v = buf_ld(rin, (((u32)j << a.logC) + seq) * 8, ((u32)o << a.logC) * 8);
        if (INV) return v;
        return gl_mul(v, preg ? preg[j + o] : pre[j + o]);
    };
    // four-step twiddles from the table: loaded by pf before the last step's loads and butterflies,
    // so the table latency hides behind them; one multiply per element instead of two
    constexpr int PERL = (1 << LOGE) / RR;
    u64 tq[PERL][RR];
    // without a table: the running product's seed and step (and 7^j2), gathered by pf as well so
    // that their latency also hides behind the last step's loads and butterflies
    u64 wq[PERL], sq[PERL], p7q[PERL];
    const u64* tab = a.t4 ? a.t4 + (INV ? 0 : ((u64)t << a.logn)) + col0 : nullptr;
    const auto rtab = buf_rsrc(tab ? tab : y);
    auto pf = [&](int q, int seq, int base, int stride) {
        if (!tab) {
            const u64 j2 = col0 + seq;
            if (INV) {
                wq[q] = tw_get(a.T, a.logn, (j2 * (u64)base) & (n - 1), true);
                sq[q] = tw_get(a.T, a.logn, (j2 * (u64)stride) & (n - 1), true);
            } else {
                // 7^j2 w_N^(j2 (t + beta base)); step w_N^(j2 beta stride) = w_n^(j2 stride)
                p7q[q] = a.T.pow7[j2];
                wq[q] = tw_get(a.T, logN, (j2 * ((u64)t + ((u64)base << a.logbeta))) & maskN, false);
                sq[q] = tw_get(a.T, a.logn, (j2 * (u64)stride) & (n - 1), false);
            }
            return;
        }
        const u32 vo = (((u32)base << a.logC) + seq) * 8;
#pragma unroll
        for (int r = 0; r < RR; r++) tq[q][r] = buf_ld(rtab, vo, ((u32)(r * stride) << a.logC) * 8);
    };
    auto stg = [&](int q, int seq, int base, int stride, u64* v) {
        const u64 j2 = col0 + seq;
        if (tab) {
            const u32 vo = (((u32)base << a.logC) + seq) * 8;
#pragma unroll
            for (int r = 0; r < RR; r++) buf_st(ry, vo, ((u32)(r * stride) << a.logC) * 8, gl_mul(v[r], tq[q][r]));
            return;
        }
        u64 w = INV ? wq[q] : gl_mul(p7q[q], wq[q]);
        const u64 step = sq[q];
        if (!INV && a.preg) {  // configs[4]-class forward pass: full tiles of 8 columns
            u64 o[RR];
#pragma unroll
            for (int r = 0; r < RR; r++) {
                o[r] = gl_mul(v[r], w);
                if (r + 1 < RR) w = gl_mul(w, step);
            }
            store_pairs<RR>(o, [&](int r) { return y + ((u64)(base + r * stride) << a.logC) + (j2 & ~1ULL); });
            return;
        }
#pragma unroll
        for (int r = 0; r < RR; r++) {
            y[((u64)(base + r * stride) << a.logC) + j2] = gl_mul(v[r], w);
            if (r + 1 < RR) w = gl_mul(w, step);
        }
    };
    pass_dft<LOGR, LOGE, INV, true, NT>(tile, logTC, ltw, ldg, stg, pf);
}

// ---------------------------------------------------------------- pass A, all cosets per block
// The beta cosets of one column tile read the same coefficients: one block loads the tile once
// (16 values per thread, kept in registers) and runs the column DFTs of every coset from them,
// refilling only the coset pre-factors between cosets. Coefficient loads drop beta-fold and their
// latency is paid once per tile instead of once per coset. Forward LDE with the four-step table,
// one first-step group per thread (256 x 16 tiles of R = 256: 16 columns).
template <int LOGR>
__global__ __launch_bounds__(256, 3) void ntt_pass_a_cos(NttArgs a) {
    constexpr int LOGT = 8, LOGE = 4, NT = 1 << LOGT, R = 1 << LOGR, PITCH = row_pitch(R);
    using PL = Plan<LOGR, LOGE>;
    constexpr int R1 = 1 << PL::FIRST_LOGR, G1 = R / R1, RR = PL::LAST_R;
    static_assert((1 << LOGE) / R1 == 1, "one first-step group per thread");
    extern __shared__ u64 lds[];
    const int logTC = (a.logC < LOGT + LOGE - LOGR) ? a.logC : LOGT + LOGE - LOGR;
    const int TC = 1 << logTC;
    u64* tile = lds;
    u64* ltw = lds + TC * PITCH;
    u64* pre = ltw + R;
    const int poly = blockIdx.y, col0 = blockIdx.x * TC;
    const u64 n = 1ULL << a.logn;
    const int beta = 1 << a.logbeta;
    const u64* pt4 = a.pt;
    const u64* pre_all = pt4 + R + (1 << a.logC);  // [t][R]
    for (int i = threadIdx.x; i < R; i += NT) {
        ltw[i] = pt4[i];
        pre[i] = pre_all[i];
    }
    // this thread's first-step group (stockham, SEQ_FAST, q = 0): its R1 coefficients, loaded once
    const int g = threadIdx.x, seq0 = g & (TC - 1), j0 = g >> logTC;
    const auto rin = buf_rsrc(a.in + (u64)poly * a.in_stride + col0);
    u64 raw[R1];
#pragma unroll
    for (int r = 0; r < R1; r++) raw[r] = buf_ld(rin, (((u32)j0 << a.logC) + seq0) * 8, ((u32)(r * G1) << a.logC) * 8);
    __syncthreads();
    for (int t = 0; t < beta; t++) {
        const int pt = poly * beta + t;
        // next coset's pre-factor, loaded now, stored after this coset's last barrier
        const u64 pre_next = (t + 1 < beta && threadIdx.x < R) ? pre_all[(t + 1) * R + threadIdx.x] : 0;
        const auto ry = buf_rsrc(a.y + (u64)pt * n + col0);
        auto ldg = [&](int, int j, int o) -> u64 { return gl_mul(raw[o / G1], pre[j + o]); };
        // the four-step twiddles are applied by pass B as it loads (a.tq_b): the intermediate is
        // stored weakly reduced, pass B's multiply canonicalises it
        auto stg = [&](int, int seq, int base, int stride, u64* v) {
            const u32 vo = (((u32)base << a.logC) + seq) * 8;
#pragma unroll
            for (int r = 0; r < RR; r++) buf_st(ry, vo, ((u32)(r * stride) << a.logC) * 8, v[r]);
        };
        pass_dft<LOGR, LOGE, false, true, NT>(tile, logTC, ltw, ldg, stg, [](int, int, int, int) {});  // ends with a barrier
        if (t + 1 < beta) {
            if (threadIdx.x < R) pre[threadIdx.x] = pre_next;
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- pass A, all cosets, shift twists
// ntt_pass_a_cos without the per-coset pre-factor multiply. The pre-factor of coset t at column
// row j1 = j0 + 16 r (first-step group j0, element r) splits as
//   7^(C j1) w_(beta R)^(t j1) = [7^(C j0) w_(beta R)^(t j0)] * [7^(16 C r) w_(16 beta)^(t r)]:
// the group factor is the same for a group's 16 elements, so it rides on the second step's twiddle
// (a per-coset [r][k] table: w_R^(r k) times the factor of group r); of the element factor, with
// t = M k + c (M = beta / 4 classes), w_(16 beta)^(t r) = w_(16 beta)^(c r) w_64^(k r), and w_64 = 2^39
// is a shift. So each class starts from the coefficients times 7^(16 C r) w_(16 beta)^(c r) (one
// multiply per element per class) and advances from coset to coset of its class by w_64^r (a
// shift multiply): one general multiply per output becomes ~3/4 shift + M/beta general.
// Cosets run class by class; every coset's column DFTs are otherwise those of ntt_pass_a_cos.
// Forward LDE with the four-step table, beta in {4, 8, 16}, R = 256 (256 x 16 tiles of 16 columns).
struct NoPf {
    __device__ void operator()(int, int, int, int) const {}
};
template <int R_>
__device__ __forceinline__ u64 mul_w64pow(u64 x) {  // x * w_64^R_ = x * 2^(39 R_ mod 192)
    constexpr int e = (39 * R_) % 192;
    if constexpr (e == 0) return x;
    else if constexpr (e < 96) return mul_pow2<e>(x);
    else return mul_pow2<e - 96>(P - x);  // 2^96 = -1; P - x is -x for any canonical x
}
__global__ __launch_bounds__(256, 4) void ntt_pass_a_cos2(NttArgs a) {
    constexpr int LOGR = 8, LOGT = 8, LOGE = 4, NT = 1 << LOGT, R = 1 << LOGR, PITCH = row_pitch(R);
    using PL = Plan<LOGR, LOGE>;
    constexpr int R1 = 1 << PL::FIRST_LOGR, G1 = R / R1, RR = PL::LAST_R;
    static_assert(R1 == 16 && G1 == 16 && RR == 16 && PL::NSTEP == 2, "16 x 16 column DFTs");
    extern __shared__ u64 lds[];
    const int logTC = (a.logC < LOGT + LOGE - LOGR) ? a.logC : LOGT + LOGE - LOGR;
    const int TC = 1 << logTC;
    u64* tile = lds;
    u64* comb = lds + TC * PITCH;  // [r][k] second-step twiddles of the current coset
    const int poly = blockIdx.y, col0 = blockIdx.x * TC;
    const u64 n = 1ULL << a.logn;
    const int beta = 1 << a.logbeta, M = beta >> 2, KP = beta / M;
    const u64* comb_all = a.pt + R + (1 << a.logC) + ((u64)R << a.logbeta);  // [t][16][16]
    const u64* scal = comb_all + ((u64)R << a.logbeta);                        // [c][16]
    const int g = threadIdx.x, seq0 = g & (TC - 1), j0 = g >> logTC;
    const auto rin = buf_rsrc(a.in + (u64)poly * a.in_stride + col0);
    u64 cnext = comb_all[threadIdx.x];  // coset 0's table (class 0, k = 0)
    for (int c = 0; c < M; c++) {
        // the coefficients are (re)loaded per class -- from L2 after the first class -- rather than
        // kept in registers: 32 VGPRs fewer, 4 waves per SIMD instead of 3
        u64 cur[R1];
#pragma unroll
        for (int r = 0; r < R1; r++) cur[r] = buf_ld(rin, (((u32)j0 << a.logC) + seq0) * 8, ((u32)(r * G1) << a.logC) * 8);
#pragma unroll
        for (int r = 0; r < R1; r++) cur[r] = gl_mul(cur[r], scal[c * R1 + r]);
        for (int k = 0; k < KP; k++) {
            const int t = M * k + c, pt = poly * beta + t;
            // (the previous coset's last step has passed its barrier; only this coset's second step,
            // behind the barrier between the two steps, reads the table)
            comb[threadIdx.x] = cnext;
            const int tn = k + 1 < KP ? t + M : c + 1;  // next coset in processing order
            if (tn < beta) cnext = comb_all[(tn << 8) + threadIdx.x];
            const auto ry = buf_rsrc(a.y + (u64)pt * n + col0);
            auto ldg = [&](int, int, int o) -> u64 { return cur[o / G1]; };
            auto stg = [&](int, int seq, int base, int stride, u64* v) {
                const u32 vo = (((u32)base << a.logC) + seq) * 8;
#pragma unroll
                for (int r = 0; r < RR; r++) buf_st(ry, vo, ((u32)(r * stride) << a.logC) * 8, v[r]);
            };
            pass_dft<LOGR, LOGE, false, true, NT, decltype(ldg), decltype(stg), NoPf, true>(tile, logTC, comb, ldg, stg,
                                                                                           NoPf{});  // ends with a barrier
            if (k + 1 < KP) static_for<R1>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                cur[r] = mul_w64pow<r>(cur[r]);
            });
        }
    }
}

// ---------------------------------------------------------------- pass A, R = 1024, no four-step table
// Forward pass A of the LDEs past the four-step tables (configs[4]: 2^20 x 16, R = C = 1024, radix
// 32 x 32): one (8-column tile, poly, coset) per 256-thread block, a tile's cosets side by side on one
// XCD (xcd_block_coset: the coefficient tile comes from HBM once, from L2 beta - 1 times).
//  * Coset pre-factor g_t^j1 (g_t = 7^C w_(beta R)^t), j1 = j0 + 32 r: the group factor g_t^j0 rides on
//    the second step's twiddle (a per-coset [r][k] table w_1024^(r k) g_t^r in LDS), the element factor
//    g_t^(32 r) on the first step's loads.
//  * Four-step factor of output k1 of column j2: 7^j2 w_N^(j2 (t + beta k1)) = s_t(j2) w_n^(j2 k1). s_t(j2)
//    = 7^j2 w_N^(j2 t) does not depend on k1, so it joins the element factor (pre2[r][seq] = g_t^(32 r)
//    s_t(col0 + seq), one multiply per thread per block), and every output takes one multiply by its
//    entry of the t-independent [k1][j2] table (8 MiB, appended to the pass tables; a column tile's 16
//    cosets read its 64 KiB slice from one L2) -- not a running product (two multiplies per output).
//  * The exchange between the two radix-32 steps goes through the LDS tile in 32-bit halves
//    (pass_dft_split at split_pitch: 42 KiB per block, three blocks per CU, no bank conflicts).
//  * The intermediate is tile-major: the block's 8 columns x 1024 rows are one contiguous 64 KiB run,
//    so rows k1, k1 + 1 of a column pair -- lanes of one store_pairs instruction -- fill whole 128 B
//    lines (row-major, each line was half-written by two blocks 16 launches apart: 15 % more write
//    requests).
__global__ __launch_bounds__(256, 3) void ntt_pass_a_r1024(NttArgs a) {
    constexpr int LOGR = 10, LOGE = 5, NT = 256, R = 1 << LOGR, RR = 32, logTC = 3, TC = 1 << logTC;
    constexpr int PITCH = split_pitch(R, LOGE, NT_LOG2(NT) + LOGE - LOGR);
    extern __shared__ u64 lds[];
    u32* tile = reinterpret_cast<u32*>(lds);
    u64* comb = lds + (TC * PITCH + 1) / 2;
    u64* pre2 = comb + R;  // [r][seq]: first-step factors of this tile's 8 columns
    int bx, by;
    xcd_block_coset(a.logbeta, bx, by);
    const int pt = by, col0 = bx * TC, poly = pt >> a.logbeta, t = pt & ((1 << a.logbeta) - 1);
    const u64 n = 1ULL << a.logn;
    const u64* pre = a.pt + R + (1 << a.logC) + (u64)t * R;                                     // g_t^j1
    const u64* comb_t = a.pt + R + (1 << a.logC) + ((u64)R << a.logbeta) + ((u64)t << LOGR);  // [r][k]
    const u64* xt = a.pt + R + (1 << a.logC) + ((u64)(2 * R) << a.logbeta);
    const u64* seed_t = xt + ((u64)t << 10);                   // [t][j2] s_t(j2)
    const u64* t4 = xt + ((u64)1 << (10 + a.logbeta));          // [k1][j2] w_n^(j2 k1)
    for (int i = threadIdx.x; i < R; i += NT) comb[i] = comb_t[i];
    // (comb is read only by the second step, behind pass_dft_split's first barrier; the first step's
    // element r of group j is row j + 32 r)
    pre2[threadIdx.x] = gl_mul(pre[(threadIdx.x >> 3) << 5], seed_t[col0 + (threadIdx.x & 7)]);
    __syncthreads();
    const auto rin = buf_rsrc(a.in + (u64)poly * a.in_stride + col0);
    auto ldg = [&](int seq, int j, int o) -> u64 {
        return gl_mul(buf_ld(rin, (((u32)j << a.logC) + seq) * 8, ((u32)o << a.logC) * 8), pre2[(o >> 5) * TC + seq]);
    };
    // tile-major intermediate: [tile][k1][8]; table [k1][j2] and intermediate through buffer resources
    // (per-lane offset in a VGPR, the r * stride part wave-uniform in the SGPR offset)
    const auto ry = buf_rsrc(a.y + (u64)pt * n + ((u64)bx << 13));
    const auto rt = buf_rsrc(t4 + col0);
    auto stg = [&](int, int seq, int base, int stride, u64* v) {
        const u32 vt = (((u32)base << 10) + seq) * 8;
        u64 tb[RR];
#pragma unroll
        for (int r = 0; r < RR; r++) tb[r] = buf_ld(rt, vt, ((u32)(r * stride) << 10) * 8);
#pragma unroll
        for (int r = 0; r < RR; r += 2) gl_mul2(v[r], tb[r], v[r + 1], tb[r + 1]);
        store_pairs_buf<RR>(v, ry, (((u32)base << 3) + (seq & ~1)) * 8, ((u32)stride << 3) * 8);
    };
    pass_dft_split<LOGR, LOGE, false, true, NT, decltype(ldg), decltype(stg), NoPf, true>(tile, logTC, comb, ldg, stg,
                                                                                       NoPf{});
}
size_t pass_a_r1024_lds() { return (size_t)((8 * split_pitch(1024, 5, 3) + 1) / 2 + 1024 + 256) * sizeof(u64); }

// Forward pass B of the same LDEs: row DFTs of C = 1024 (radix 32 x 32), one 8-row tile per 256-thread
// block with the exchange in 32-bit halves (three blocks per CU). The first step walks the tile-major
// intermediate rows fastest (8 rows x 8 columns of one column tile = 512 contiguous bytes per load
// instruction); canonical outputs are stored as row pairs (store_pairs) into the coset-major LDE.
__global__ __launch_bounds__(256, 3) void ntt_pass_b_r1024(NttArgs a) {
    constexpr int LOGC = 10, LOGE = 5, NT = 256, C = 1 << LOGC, R1 = 32, G1 = C / R1, RR = 32, logTR = 3;
    constexpr int TR = 1 << logTR, PITCH = split_pitch(C, LOGE, logTR);
    extern __shared__ u64 lds[];
    u32* tile = reinterpret_cast<u32*>(lds);
    u64* ltw = lds + (TR * PITCH + 1) / 2;
    int bx, by;
    xcd_block(true, bx, by);
    const int pt = by, k10 = bx * TR;
    const u64 n = 1ULL << a.logn;
    for (int i = threadIdx.x; i < C; i += NT) ltw[i] = a.pt[(1 << a.logR) + i];
    // this thread's first-step group (stockham, SEQ_FAST): row seq0 of the tile, columns j0 + 32 r
    const int seq0 = threadIdx.x & (TR - 1), j0 = threadIdx.x >> logTR;
    const auto ry = buf_rsrc(a.y + (u64)pt * n);
    const u32 vy = ((((u32)(j0 >> 3)) << 13) + ((u32)(k10 + seq0) << 3) + (j0 & 7)) * 8;
    u64 yv[R1];
#pragma unroll
    for (int r = 0; r < R1; r++) yv[r] = buf_ld(ry, vy, ((u32)r << 15) * 8);  // column j0 + 32 r: 4 tiles further
    __syncthreads();
    auto ldg = [&](int, int, int o) -> u64 { return yv[o / G1]; };
    const auto ro = buf_rsrc(a.out + (u64)pt * n + k10);
    auto stg = [&](int, int seq, int base, int stride, u64* v) {  // the last butterfly level made v canonical
        store_pairs_buf<RR>(v, ro, ((u32)(seq & ~1) + ((u32)base << a.logR)) * 8, ((u32)stride << a.logR) * 8);
    };
    pass_dft_split<LOGC, LOGE, false, true, NT, decltype(ldg), decltype(stg), NoPf, false, true>(tile, logTR, ltw, ldg, stg,
                                                                                              NoPf{});
}
size_t pass_b_r1024_lds() { return (size_t)((8 * split_pitch(1024, 5, 3) + 1) / 2 + 1024) * sizeof(u64); }

// ---------------------------------------------------------------- pass B: row DFTs (size C)
template <int LOGC, bool INV, int LOGT, int LOGE>
__global__ __launch_bounds__(1 << LOGT) void ntt_pass_b(NttArgs a) {
    constexpr int C = 1 << LOGC, RR = Plan<LOGC, LOGE>::LAST_R, NT = 1 << LOGT;
    extern __shared__ u64 lds[];
    const int logTR = (a.logR < LOGT + LOGE - LOGC) ? a.logR : LOGT + LOGE - LOGC;
    const int TR = 1 << logTR;
    u64* tile = lds;
    u64* ltw = lds + TR * row_pitch(C, LOGE, LOGT + LOGE - LOGC);
    int bx, by;
    xcd_block(a.xcd & 2, bx, by);
    const int pt = by, k10 = bx * TR;
    const u64 n = 1ULL << a.logn;
    if (a.pt) {
        const u64* pt4 = a.pt + (1 << a.logR);
        for (int i = threadIdx.x; i < C; i += NT) ltw[i] = pt4[i];
    } else {
        for (int i = threadIdx.x; i < C; i += NT) ltw[i] = tw_get(a.T, LOGC, i, INV);
    }
    __syncthreads();
    const u64* y = a.y + (u64)pt * n;
    // four-step twiddles at the load when pass A left them out (a.tq_b): the table has the
    // intermediate's [k1][j2] layout, so its loads are as coalesced as the data's
    const u64* tqb = (!INV && a.tq_b) ? a.t4 + ((u64)(pt & ((1 << a.logbeta) - 1)) << a.logn) : nullptr;
    // with the twiddles, all of a thread's first-step loads (data and table) are issued before the
    // first multiply (a load next to its multiply would be waited for one at a time: the field
    // primitives are asm statements the scheduler does not move loads across). One first-step group
    // per thread, lanes along the row (multi-step rows of 16-element threads).
    using PLB = Plan<LOGC, LOGE>;
    constexpr int R1 = 1 << PLB::FIRST_LOGR, G1 = C / R1;
    constexpr bool PRE = !INV && PLB::NSTEP > 1 && (1 << LOGE) == R1;
    u64 yv[PRE ? R1 : 1], tv[PRE ? R1 : 1];
    if constexpr (PRE) {
        if (tqb) {
            const int seq0 = threadIdx.x / G1, j0 = threadIdx.x % G1;
            const u64 i0 = ((u64)(k10 + seq0) << LOGC) + j0;
#pragma unroll
            for (int r = 0; r < R1; r++) {
                yv[r] = y[i0 + r * G1];
                tv[r] = tqb[i0 + r * G1];
            }
        }
    }
    auto ldg = [&](int seq, int j, int o) -> u64 {
        if constexpr (PRE) {
            if (tqb) return gl_mul(yv[o / G1], tv[o / G1]);
        }
        const u64 i = ((u64)(k10 + seq) << LOGC) + j + o;
        return tqb ? gl_mul(y[i], tqb[i]) : y[i];
    };
    const auto rout = buf_rsrc(a.out + (u64)pt * n + k10);
    auto stg = [&](int, int seq, int base, int stride, u64* v) {
#pragma unroll
        for (int r = 0; r < RR; r++) {
            const u64 k = (u64)(k10 + seq) + ((u64)(base + r * stride) << a.logR);
            if (INV) {
                if (k < a.keep) {
                    u64 x = a.t4 ? canon(v[r]) : gl_mul(v[r], a.scale);  // the table carries 1/n
                    if (a.off7) x = gl_mul(x, a.T.ipow7[k]);
                    a.out[(u64)pt * a.out_stride + k] = x;
                }
            } else {
                // pt = poly * beta + t -> coset-major; k - k10 = seq + (base + r stride) R
                buf_st(rout, (seq + ((u32)base << a.logR)) * 8, ((u32)(r * stride) << a.logR) * 8, canon(v[r]));
            }
        }
    };
    // multi-step rows: first step along the row (coalesced loads); one-step rows: lanes along
    // sequences so the (final) global store is coalesced
    pass_dft<LOGC, LOGE, INV, (Plan<LOGC, LOGE>::NSTEP == 1), NT>(tile, logTR, ltw, ldg, stg,
                                                                   [](int, int, int, int) {});
}

// ---------------------------------------------------------------- pass B, forward with the four-step table
// ntt_pass_b specialised to the path every tabled LDE takes (the all-coset pass A left the four-step
// twiddles to it): one first-step group per thread, data and table loaded up front, no run-time
// branches for the other paths; the exchange between its two steps goes through the LDS tile in
// 32-bit halves (pass_dft_split)
template <int LOGC, int LOGT, int LOGE>
__global__ __launch_bounds__(1 << LOGT) void ntt_pass_b_tq(NttArgs a) {
    constexpr int C = 1 << LOGC, RR = Plan<LOGC, LOGE>::LAST_R, NT = 1 << LOGT;
    using PLB = Plan<LOGC, LOGE>;
    constexpr int R1 = 1 << PLB::FIRST_LOGR, G1 = C / R1;
    static_assert(PLB::NSTEP > 1 && (1 << LOGE) == R1, "one full-radix first-step group per thread");
    extern __shared__ u64 lds[];
    const int logTR = (a.logR < LOGT + LOGE - LOGC) ? a.logR : LOGT + LOGE - LOGC;
    const int TR = 1 << logTR;
    u64* tile = lds;
    const int tw = TR * row_pitch(C, LOGE, LOGT + LOGE - LOGC);
    u64* ltw = reinterpret_cast<u64*>(reinterpret_cast<u32*>(lds) + tw);
    int bx, by;
    xcd_block(a.xcd & 2, bx, by);
    const int pt = by, k10 = bx * TR;
    const u64 n = 1ULL << a.logn;
    {
        // the second step's twiddles as an [r][k] table (w_C^(r k), r, k < 16): each read is a fixed
        // LDS offset r * 128 from the lane's k * 8, so no per-element address arithmetic (w_C[r k]
        // needs a multiply and an add per element)
        static_assert(LOGC == 2 * LOGE, "two full-radix steps");
        const u64* pt4 = a.pt + (1 << a.logR);
        for (int i = threadIdx.x; i < C; i += NT) ltw[i] = pt4[(i >> LOGE) * (i & ((1 << LOGE) - 1))];
    }
    const int seq0 = threadIdx.x / G1, j0 = threadIdx.x % G1;
    const u64 i0 = ((u64)(k10 + seq0) << LOGC) + j0;
    const u64* y = a.y + (u64)pt * n + i0;
    const u64* tq = a.t4 + ((u64)(pt & ((1 << a.logbeta) - 1)) << a.logn) + i0;
    u64 yv[R1], tv[R1];
#pragma unroll
    for (int r = 0; r < R1; r++) {
        yv[r] = y[r * G1];
        tv[r] = tq[r * G1];
    }
    __syncthreads();
    auto ldg = [&](int, int, int o) -> u64 { return gl_mul(yv[o / G1], tv[o / G1]); };
    const auto rout = buf_rsrc(a.out + (u64)pt * n + k10);
    auto stg = [&](int, int seq, int base, int stride, u64* v) {  // the last butterfly level made v canonical
        // (16-byte paired stores, store_pairs_buf, measured neutral here: profiles/r05/tqp_ab.txt)
#pragma unroll
        for (int r = 0; r < RR; r++)
            buf_st(rout, (seq + ((u32)base << a.logR)) * 8, ((u32)(r * stride) << a.logR) * 8, v[r]);
    };
    pass_dft_split<LOGC, LOGE, false, false, NT, decltype(ldg), decltype(stg), NoPf, true, true>(
        reinterpret_cast<u32*>(tile), logTR, ltw, ldg, stg, NoPf{});
}

// ---------------------------------------------------------------- pass B, persistent (forward, no table)
// The row DFTs of an LDE past the four-step tables (configs[4]: 2^24 points, radix 32 x 32, 8 rows
// per tile, two blocks per CU). One tile per block waited on its loads for 48 % of its wave cycles
// (profiles/r02/lde_pmc_2p16_vs_2p20.json): here a block loops over its share of the (row tile,
// poly-coset) tiles and issues the next tile's first-step loads into registers before it
// transforms the current one, so one tile's loads are in flight during the other's butterflies.
// Tiles are dealt per XCD in contiguous ranges (the blocks of XCD x = blockIdx % 8 walk the x-th
// eighth of the tiles side by side), so the 64-byte output runs of neighbouring tiles meet in
// one L2, as xcd_block arranges for the one-tile form.
template <int LOGC, int LOGT, int LOGE, int MINW>
__global__ __launch_bounds__(1 << LOGT, MINW) void ntt_pass_b_pers(NttArgs a, int ntx, int ntiles) {
    constexpr int C = 1 << LOGC, RR = Plan<LOGC, LOGE>::LAST_R, NT = 1 << LOGT;
    using PLB = Plan<LOGC, LOGE>;
    constexpr int R1 = 1 << PLB::FIRST_LOGR, G1 = C / R1;
    static_assert(PLB::NSTEP > 1 && (1 << LOGE) == R1, "one full-radix first-step group per thread");
    constexpr int logTR = LOGT + LOGE - LOGC, TR = 1 << logTR;
    extern __shared__ u64 lds[];
    u64* tile = lds;
    u64* ltw = lds + TR * row_pitch(C, LOGE, logTR);
    {
        const u64* pt4 = a.pt + (1 << a.logR);
        for (int i = threadIdx.x; i < C; i += NT) ltw[i] = pt4[i];
    }
    __syncthreads();
    const u64 n = 1ULL << a.logn;
    const int per_x = gridDim.x >> 3, x = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int span = (ntiles + 7) >> 3, tend = min((x + 1) * span, ntiles);
    const int seq0 = threadIdx.x / G1, j0 = threadIdx.x % G1;
    auto load = [&](int ti, u64* dst) {
        const int pt = ti / ntx, k10 = (ti - pt * ntx) * TR;
        const u64* y = a.y + (u64)pt * n + ((u64)(k10 + seq0) << LOGC) + j0;
#pragma unroll
        for (int r = 0; r < R1; r++) dst[r] = y[r * G1];
    };
    int ti = x * span + slot;
    u64 yv[R1];
    if (ti < tend) load(ti, yv);
    for (; ti < tend; ti += per_x) {
        const int pt = ti / ntx, k10 = (ti - pt * ntx) * TR;
        u64 nx[R1];
        if (ti + per_x < tend) load(ti + per_x, nx);
        auto ldg = [&](int, int, int o) -> u64 { return yv[o / G1]; };
        u64* out = a.out + (u64)pt * n + k10;
        auto stg = [&](int, int seq, int base, int stride, u64* v) {
            u64 o[RR];
#pragma unroll
            for (int r = 0; r < RR; r++) o[r] = canon(v[r]);
            store_pairs<RR>(o, [&](int r) { return out + (seq & ~1) + ((u64)(base + r * stride) << a.logR); });
        };
        pass_dft<LOGC, LOGE, false, false, NT>(tile, logTR, ltw, ldg, stg, [](int, int, int, int) {});
#pragma unroll
        for (int r = 0; r < R1; r++) yv[r] = nx[r];
    }
}

// ---------------------------------------------------------------- dispatch
// tiles above 64 KiB of LDS need the per-kernel opt-in (a workgroup may use 160 KiB on gfx950)
#define XFG_NTT_LAUNCH(KERNEL, NT)                                                                          \
    do {                                                                                                    \
        if (lds > 65536) {                                                                                  \
            static const bool ok_ = hipFuncSetAttribute((const void*)KERNEL,                                \
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                                        160 * 1024) == hipSuccess;                          \
            (void)ok_;                                                                                      \
        }                                                                                                   \
        hipLaunchKernelGGL(KERNEL, g, dim3(NT), lds, s, a);                                                 \
    } while (0)
template <bool INV>
static void run_pass_a(int logR, int logT, int logE, dim3 g, size_t lds, hipStream_t s, const NttArgs& a) {
#define XFG_CASE_A(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_a<L, INV, 8, 4>), 256); break;
#define XFG_CASE_A10(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_a<L, INV, 10, 4>), 1024); break;
#define XFG_CASE_A9(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_a<L, INV, 9, 4>), 512); break;
#define XFG_CASE_A5(L, T) \
    case L: XFG_NTT_LAUNCH((ntt_pass_a<L, INV, T, 5>), (1 << T)); break;
    if (logE == 5) {
        if (logT == 9) {
            switch (logR) {
                XFG_CASE_A5(9, 9) XFG_CASE_A5(10, 9)
                default: break;
            }
        } else {
            switch (logR) {
                XFG_CASE_A5(9, 8) XFG_CASE_A5(10, 8)
                default: break;
            }
        }
        return;
    }
    if (logT == 10) {
        switch (logR) {
            XFG_CASE_A10(9) XFG_CASE_A10(10)
            default: break;
        }
        return;
    }
    if (logT == 9) {
        switch (logR) {
            XFG_CASE_A9(9) XFG_CASE_A9(10)
            default: break;
        }
        return;
    }
    switch (logR) {
        XFG_CASE_A(1) XFG_CASE_A(2) XFG_CASE_A(3) XFG_CASE_A(4) XFG_CASE_A(5) XFG_CASE_A(6)
        XFG_CASE_A(7) XFG_CASE_A(8) XFG_CASE_A(9) XFG_CASE_A(10)
        default: break;
    }
#undef XFG_CASE_A
#undef XFG_CASE_A10
#undef XFG_CASE_A9
#undef XFG_CASE_A5
}
template <bool INV>
static void run_pass_b(int logC, int logT, int logE, dim3 g, size_t lds, hipStream_t s, const NttArgs& a) {
#define XFG_CASE_B(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_b<L, INV, 8, 4>), 256); break;
#define XFG_CASE_B10(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_b<L, INV, 10, 4>), 1024); break;
#define XFG_CASE_B9(L) \
    case L: XFG_NTT_LAUNCH((ntt_pass_b<L, INV, 9, 4>), 512); break;
#define XFG_CASE_B5(L, T) \
    case L: XFG_NTT_LAUNCH((ntt_pass_b<L, INV, T, 5>), (1 << T)); break;
    if (logE == 5) {
        if (logT == 9) {
            switch (logC) {
                XFG_CASE_B5(9, 9) XFG_CASE_B5(10, 9)
                default: break;
            }
        } else {
            switch (logC) {
                XFG_CASE_B5(9, 8) XFG_CASE_B5(10, 8)
                default: break;
            }
        }
        return;
    }
    if (logT == 10) {
        switch (logC) {
            XFG_CASE_B10(9) XFG_CASE_B10(10) XFG_CASE_B10(11)
            default: break;
        }
        return;
    }
    if (logT == 9) {
        switch (logC) {
            XFG_CASE_B9(9) XFG_CASE_B9(10) XFG_CASE_B9(11)
            default: break;
        }
        return;
    }
    switch (logC) {
        XFG_CASE_B(2) XFG_CASE_B(3) XFG_CASE_B(4) XFG_CASE_B(5) XFG_CASE_B(6) XFG_CASE_B(7)
        XFG_CASE_B(8) XFG_CASE_B(9) XFG_CASE_B(10) XFG_CASE_B(11) XFG_CASE_B(12)
        default: break;
    }
#undef XFG_CASE_B
#undef XFG_CASE_B10
#undef XFG_CASE_B9
#undef XFG_CASE_B5
}
#undef XFG_NTT_LAUNCH

// split n = R * C: evenly below 2^18, C = 2R from 2^18 on except 2^20 (faster at 2^18; see
// scripts/ntt_split.py; at 2^24 the splits C = 512 / 2048 / 4096 measured slower than 1024)
static void ntt_split(int logn, int& logR, int& logC) {
    if (logn >= 18) {
        logC = logn == 20 ? 10 : logn / 2 + 1;  // 2^20: R = C = 1024, both passes wide-tiled (3 % faster)
    } else {
        logC = logn - logn / 2;
    }
    logR = logn - logC;
}

__global__ void fourstep_kernel(u64* out, int logn, int logbeta, int logC, u64 scale, Tables T) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 n = 1ULL << logn;
    if (logbeta < 0) {
        if (i >= n) return;
        const u64 k1 = i >> logC, j2 = i & ((1ULL << logC) - 1);
        out[i] = gl_mul(tw_get(T, logn, (j2 * k1) & (n - 1), true), scale);
    } else {
        const int logN = logn + logbeta;
        if (i >= (1ULL << logN)) return;
        const u64 t = i >> logn, k1 = (i & (n - 1)) >> logC, j2 = i & ((1ULL << logC) - 1);
        out[i] = gl_mul(T.pow7[j2], tw_get(T, logN, (j2 * (t + (k1 << logbeta))) & ((1ULL << logN) - 1), false));
    }
}
// pass tables appended to a four-step table: w_R^(+-i) (i < R), w_C^(+-i) (i < C), and for the
// forward LDE the coset pre-factors 7^(C i) w_(beta R)^(t i) at [t][i] -- what every pass block
// would otherwise gather from the master tables at its start
__global__ void pass_tables_kernel(u64* out, int logn, int logbeta, int logR, int logC, Tables T) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 R = 1ULL << logR, C = 1ULL << logC;
    const bool inv = logbeta < 0;
    if (i < R) {
        out[i] = tw_get(T, logR, i, inv);
    } else if (i < R + C) {
        out[i] = tw_get(T, logC, i - R, inv);
    } else if (!inv && i < R + C + (R << logbeta)) {
        const u64 t = (i - R - C) >> logR, j = (i - R - C) & (R - 1);
        out[i] = gl_mul(T.pow7[j << logC], tw_get(T, logR + logbeta, (t * j) & ((1ULL << (logR + logbeta)) - 1), false));
    } else if (!inv && logR == 10 && i < R + C + 2 * (R << logbeta)) {
        // ntt_pass_a_r1024: [t][r][k] = w_1024^(r k) g_t^r, g_t^r = 7^(C r) w_(beta R)^(t r)  (r, k < 32)
        const u64 q = i - R - C - (R << logbeta);
        const u64 t = q >> 10, r = (q >> 5) & 31, k = q & 31;
        const u64 g = gl_mul(T.pow7[r << logC], tw_get(T, logR + logbeta, (t * r) & ((1ULL << (logR + logbeta)) - 1), false));
        out[i] = gl_mul(tw_get(T, logR, r * k, false), g);
    } else if (!inv && logR == 10 && i < R + C + 2 * (R << logbeta) + (C << logbeta) + R * C) {
        // ntt_pass_a_r1024's four-step factors: [t][j2] 7^j2 w_N^(j2 t) (t < beta, j2 < C) and the
        // t-independent four-step table [k1][j2] w_n^(j2 k1) (R x C)
        const u64 q = i - R - C - 2 * (R << logbeta);
        const int logn = logR + logC, logN = logn + logbeta;
        if (q < (C << logbeta)) {
            const u64 t = q >> logC, j2 = q & (C - 1);
            out[i] = gl_mul(T.pow7[j2], tw_get(T, logN, (j2 * t) & ((1ULL << logN) - 1), false));
        } else {
            const u64 k1 = (q - (C << logbeta)) >> logC, j2 = q & (C - 1);
            out[i] = tw_get(T, logn, (j2 * k1) & ((1ULL << logn) - 1), false);
        }
    } else if (!inv && logR == 8 && logbeta >= 2) {
        // ntt_pass_a_cos2: [t][r][k] = w_R^(r k) 7^(C r) w_(beta R)^(t r), then [c][r] = 7^(16 C r) w_(16 beta)^(c r)
        const u64 q = i - R - C - (R << logbeta);
        const u64 M = 1ULL << (logbeta - 2);
        if (q < (R << logbeta)) {
            const u64 t = q >> 8, r = (q >> 4) & 15, k = q & 15;
            const u64 grp = gl_mul(T.pow7[r << logC], tw_get(T, logR + logbeta, (t * r) & ((1ULL << (logR + logbeta)) - 1), false));
            out[i] = gl_mul(tw_get(T, logR, r * k, false), grp);
        } else if (q < (R << logbeta) + 16 * M) {
            const u64 c = (q - (R << logbeta)) >> 4, r = q & 15;
            out[i] = gl_mul(T.pow7[(16 * r) << logC], tw_get(T, 4 + logbeta, (c * r) & ((1ULL << (4 + logbeta)) - 1), false));
        }
    }
}
// entries of the ntt_pass_a_cos2 tables appended to the forward pass tables (R = 256, beta >= 4), or of
// the ntt_pass_a_r1024 tables (R = 1024)
static u64 cos2_extra(int logR, int logC, int logbeta) {
    if (logbeta >= 0 && logR == 10 && logC == 10) return (1ULL << (logR + logbeta)) + (1ULL << (logC + logbeta)) + (1ULL << (logR + logC));
    return (logbeta >= 0 && logR == 8 && logbeta >= 2) ? ((1ULL << (logR + logbeta)) + (16ULL << (logbeta - 2))) : 0;
}
u64 pass_tables_size(int logn, int logbeta) {
    int logR, logC;
    ntt_split(logn, logR, logC);
    return (1ULL << logR) + (1ULL << logC) + (logbeta >= 0 ? (1ULL << (logR + logbeta)) : 0) + cos2_extra(logR, logC, logbeta);
}
void build_pass_tables(u64* out, int logn, int logbeta, const Tables& T, hipStream_t s) {
    int logR, logC;
    ntt_split(logn, logR, logC);
    const u64 cnt = pass_tables_size(logn, logbeta);
    hipLaunchKernelGGL(pass_tables_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, out, logn, logbeta,
                       logR, logC, T);
}
__host__ __device__ u64 fourstep_main(int logn, int logbeta) { return 1ULL << (logn + (logbeta > 0 ? logbeta : 0)); }
u64 fourstep_size(int logn, int logbeta) {
    int logR, logC;
    ntt_split(logn, logR, logC);
    return fourstep_main(logn, logbeta) + (1ULL << logR) + (1ULL << logC) + (logbeta >= 0 ? (1ULL << (logR + logbeta)) : 0) +
           cos2_extra(logR, logC, logbeta);
}
void build_fourstep(u64* out, int logn, int logbeta, const Tables& T, hipStream_t s) {
    int logR, logC;
    ntt_split(logn, logR, logC);
    const u64 cnt = fourstep_main(logn, logbeta), extra = fourstep_size(logn, logbeta) - cnt;
    hipLaunchKernelGGL(fourstep_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, out, logn, logbeta, logC,
                       gl_inv(1ULL << logn), T);
    hipLaunchKernelGGL(pass_tables_kernel, dim3((unsigned)((extra + 255) / 256)), dim3(256), 0, s, out + cnt, logn,
                       logbeta, logR, logC, T);
}

static void ntt_run(NttArgs& a, int npoly, bool inv, hipStream_t s) {
    ntt_split(a.logn, a.logR, a.logC);
    const int R = 1 << a.logR, C = 1 << a.logC;
    // Pass shapes (the alternatives named there measured slower on the box):
    // * radix-32 steps (32 elements per thread) for pass sizes 2^9 and 2^10: 16 x 32 and 32 x 32
    //   instead of 2 x 16 x 16 and 4 x 16 x 16, one general-twiddle step fewer;
    // * wide tiles (1024 threads, 16384 elements) where a 4096-element radix-16 tile would hold fewer
    //   than 16 columns (pass A, R >= 512) or rows (pass B, C >= 512), so the scattered stores write
    //   whole 128 B lines; pass B at C <= 1024 runs 512-thread blocks (8192 elements, <= 78 KiB, two
    //   blocks per CU: one block's barriers and loads hide behind the other's butterflies);
    // * radix-32 tiles: pass A 16 columns (512 threads at R = 1024, 256 at R = 512; the forward
    //   R = 1024 pass past the four-step tables at other C, e.g. 2^21, 256 threads x 8 columns with the
    //   coset pre-factors read from L2 -- 76 KiB of LDS, two blocks per CU), pass B 8192 elements (256
    //   threads, two blocks per CU). configs[4]'s 2^20 takes the dedicated R = C = 1024 passes below.
    const int eA = (a.logR >= 9 && a.logR <= 10 && a.logC >= 4) ? 5 : 4;
    const int eB = (a.logC >= 9 && a.logC <= 10 && a.logR >= 3) ? 5 : 4;
    const bool capA = a.logR >= 9 && a.logR <= 10 && a.logC >= 4, capB = a.logC >= 9 && a.logC <= 11 && a.logR >= 4;
    int ltA = capA ? 10 : 8;
    int ltB = capB ? (a.logC <= 10 ? 9 : 10) : 8;
    if (eA == 5) ltA = (!inv && a.logR == 10 && a.pt) ? 8 : a.logR - 1;
    if (eB == 5) ltB = 8;
    const int logTC = a.logC < ltA + eA - a.logR ? a.logC : ltA + eA - a.logR;
    const int logTR = a.logR < ltB + eB - a.logC ? a.logR : ltB + eB - a.logC;
    const int ncos = inv ? 1 : (1 << a.logbeta);
    a.preg = (!inv && a.pt && eA == 5 && ltA == 8 && a.logR == 10) ? 1 : 0;
    size_t lds_a = ((size_t)(1 << logTC) * row_pitch(R, eA, ltA + eA - a.logR) + (a.preg ? 1 : 2) * R) * sizeof(u64);
    size_t lds_b = ((size_t)(1 << logTR) * row_pitch(C, eB, ltB + eB - a.logC) + C) * sizeof(u64);
    dim3 ga(C >> logTC, npoly * ncos), gb(R >> logTR, npoly * ncos);
    // XCD-contiguous block order where a tile row of the scattered writes is narrower than a 128 B
    // line: pass A stores TC consecutive words per row, pass B TR (xcd_block)
    a.xcd = (logTC < 4 ? 1 : 0) | (logTR < 4 ? 2 : 0) | (a.preg ? 4 : 0);
    if (inv) {
        run_pass_a<true>(a.logR, ltA, eA, ga, lds_a, s, a);
        run_pass_b<true>(a.logC, ltB, eB, gb, lds_b, s, a);
        return;
    }
    if (!a.t4 && a.pt && a.logR == 10 && a.logC == 10 && eA == 5 && eB == 5) {
        // past the four-step tables at n = 2^20 (configs[4])
        const size_t la = pass_a_r1024_lds(), lb = pass_b_r1024_lds();
        hipLaunchKernelGGL(ntt_pass_a_r1024, dim3(C >> 3, npoly << a.logbeta), dim3(256), la, s, a);
        hipLaunchKernelGGL(ntt_pass_b_r1024, dim3(R >> 3, npoly << a.logbeta), dim3(256), lb, s, a);
        return;
    }
    // pass A: all cosets of a column tile in one block where the four-step table exists (R = 256):
    // shift-twisted cosets (ntt_pass_a_cos2) for beta >= 4, per-coset pre-factors (ntt_pass_a_cos) at
    // beta = 2; the four-step twiddles are then applied by pass B as it loads (tq_b). Only for launch
    // sets of >= 512 such blocks (two per CU): the all-coset grid is C / 16 blocks per polynomial, so
    // a small set (one proof's trace: 7 polynomials, its composition or DEEP column: 1) leaves most CUs
    // idle while each block walks its beta cosets, and one block per (tile, poly, coset) -- ntt_pass_a,
    // beta times the grid -- finishes sooner: 2^16 x 8, 1 / 7 / 16 / 28 polynomials 52 / 67 / 77 / 110 us
    // against 20 / 41 / 66 / 107 us; 32 / 64 / 224 polynomials 119 / 232 / 727 against 122 / 255 / 821
    // (profiles/r06/lde_small.txt)
    if (a.t4 && a.logR == 8 && ltA == 8 && eA == 4 && !(a.xcd & 1) && (u64)npoly * (C >> logTC) >= 512) {
        a.tq_b = 1;
        if (a.logbeta >= 2)
            hipLaunchKernelGGL(ntt_pass_a_cos2, dim3(C >> logTC, npoly), dim3(256), lds_a, s, a);
        else
            hipLaunchKernelGGL(ntt_pass_a_cos<8>, dim3(C >> logTC, npoly), dim3(256), lds_a, s, a);
    } else {
        run_pass_a<false>(a.logR, ltA, eA, ga, lds_a, s, a);
    }
    if (eB == 5 && ltB == 8 && a.logC == 10 && a.logR >= 3 && !a.tq_b && a.pt) {
        // past the four-step tables: persistent pass B (prefetches the next tile during this one)
        static int cus = [] {
            int dev = 0, n = 256;
            if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
            return n;
        }();
        const int ntx = R >> logTR, ntiles = ntx * npoly * ncos;
        const int nb = std::max(8, std::min(2 * cus, ntiles) & ~7);
        hipLaunchKernelGGL((ntt_pass_b_pers<10, 8, 5, 2>), dim3(nb), dim3(256), lds_b, s, a, ntx, ntiles);
    } else if (eB == 4 && ltB == 8 && a.logC == 8 && a.logR >= 4 && a.t4 && a.tq_b && a.pt) {
        // the tabled LDE's pass B with the 32-bit split exchange (pass_dft_split): 19.5 instead of 37
        // KiB of LDS per block, 6 instead of 4 waves per SIMD (pass B 919-942 vs 946-961 us per 64-proof
        // launch set, same box)
        const size_t l = ((size_t)(1 << logTR) * row_pitch(C, 4, 4) * 4 + C * 8);
        hipLaunchKernelGGL((ntt_pass_b_tq<8, 8, 4>), gb, dim3(256), l, s, a);
    } else {
        run_pass_b<false>(a.logC, ltB, eB, gb, lds_b, s, a);
    }
}

void launch_lde(const u64* coef, u64 coef_stride, u64* out, u64* scratch, int npoly, int logn, int logbeta,
                const Tables& T, hipStream_t s) {
    NttArgs a{};
    a.in = coef;
    a.in_stride = coef_stride;
    a.y = scratch;
    a.out = out;
    a.logn = logn;
    a.logbeta = logbeta;
    a.T = T;
    a.t4 = (T.fs && logn <= FOURSTEP_MAX_LOG && logbeta <= 4) ? T.fs->fwd[logn][logbeta] : nullptr;
    a.pt = a.t4 ? a.t4 + fourstep_main(logn, logbeta)
                : ((T.fs && logn <= PASS_MAX_LOG && logbeta <= 4) ? T.fs->pass_fwd[logn][logbeta] : nullptr);
    ntt_run(a, npoly, false, s);
}

void launch_interpolate(const u64* evals, u64 in_stride, u64* out, u64 out_stride, u64* scratch, int npoly, int logn,
                        bool off7, u64 keep, const Tables& T, hipStream_t s) {
    NttArgs a{};
    a.in = evals;
    a.in_stride = in_stride;
    a.y = scratch;
    a.out = out;
    a.out_stride = out_stride;
    a.logn = logn;
    a.logbeta = 0;
    a.off7 = off7 ? 1 : 0;
    a.keep = keep;
    a.T = T;
    a.scale = gl_inv(1ULL << logn);
    a.t4 = (T.fs && logn <= FOURSTEP_MAX_LOG) ? T.fs->inv[logn] : nullptr;
    a.pt = a.t4 ? a.t4 + fourstep_main(logn, -1) : nullptr;
    ntt_run(a, npoly, true, s);
}

__global__ void field_op_kernel(int op, const u64* a, const u64* b, u64* out, u64 count) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 x = a[i], y = b[i];
    u64 r = 0;
    switch (op) {
        case 0: r = gl_mul(x, y); break;
        case 1: r = gl_add(x, y); break;
        case 2: r = gl_sub(x, y); break;
        case 3: r = gl_canon(x); break;
        case 4: {
            const int sh = (int)(y % 96);
            static_for<96>([&](auto sc) {
                if (sh == decltype(sc)::value) r = mul_pow2<decltype(sc)::value>(x);
            });
            break;
        }
        case 5: r = gl_fold(x, (u32)y); break;
        case 6: r = gl_sub_weak(x, y); break;
        case 7: r = add_w(x, y); break;
        case 8: {  // gl_mul2: both products (x y and y x) must equal; the first is returned
            u64 p = x, q = y;
            gl_mul2(p, y, q, x);
            r = p == q ? p : ~0ULL;
            break;
        }
        default: break;
    }
    out[i] = r;
}
void launch_field_op(int op, const u64* a, const u64* b, u64* out, u64 count, hipStream_t s) {
    hipLaunchKernelGGL(field_op_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, op, a, b, out, count);
}

}  // namespace xfg
