// Launch wrappers for the burn-proof STARK kernels (gfx950). Every wrapper enqueues on the given
// stream and never synchronises; batch dimension = number of independent proofs.
#pragma once
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "blake3.hpp"

namespace xfg {

// per-proof AIR constants (reference src/burn_mint_air.rs:54-71 order + Keccak constants)
struct AirConst {
    u64 pub[12];
    u64 nullifier;
    u64 commitment;
    u64 pad[2];
};

// per-proof DEEP parameters, every value an element of E (2 coordinates; the second is 0 without
// a field extension): trace coefficients a_i, composition coefficient, OOD points and the
// constant terms c1 = sum a_i T_i(z) + gamma H(z), c2 = sum a_i T_i(z g)
struct DeepParams {
    u64 a[7][2];
    u64 gamma[2];
    u64 z[2], zg[2], zinv[2], zginv[2];
    u64 c1[2], c2[2];
    u64 pad[2];
};

// precomputed four-step twiddles (ntt.hip build_fourstep): fwd[logn][logbeta] holds
// 7^j2 w_N^(j2 (t + beta k1)) at [t][k1][j2], inv[logn] holds w_n^-(j2 k1) / n at [k1][j2];
// nullptr -> the kernels form them as running products
constexpr int FOURSTEP_MAX_LOG = 22;
// forward sizes past FOURSTEP_MAX_LOG (configs[4]: 2^20 x 16 = 2^24 points, where a full table would
// be 128 MB) get no beta n table, only the per-size pass tables as one contiguous block,
// pass_fwd[logn][logbeta]: w_R^i, w_C^i and the coset pre-factors (R + C + beta R entries); at
// R = C = 1024 also the per-coset [r][k] and [t][j2] factors and the coset-independent [k1][j2]
// four-step table (8 MiB, ntt_pass_a_r1024); other sizes keep running-product four-step twiddles
constexpr int PASS_MAX_LOG = 24;
struct FourStep {
    const u64* fwd[FOURSTEP_MAX_LOG + 1][5] = {};
    const u64* inv[FOURSTEP_MAX_LOG + 1] = {};
    const u64* pass_fwd[PASS_MAX_LOG + 1][5] = {};
};
struct Tables {
    const u64* tw;     // tw[e] = w_{2^LM}^e, e < 2^LM
    int LM;
    const u64* pow7;   // 7^j,  j < 2^LM
    const u64* ipow7;  // 7^-j, j < 2^LM
    const FourStep* fs;  // host-side table registry (never dereferenced on the device)
};

// ---- NTT (four-step, natural order in/out) ----
// forward LDE: coef[poly][n] -> out[poly][beta][n] (coset-major: out[p][t][m] = P(7 w_N^(t + beta m)))
void launch_lde(const u64* coef, u64 coef_stride, u64* out, u64* scratch, int npoly, int logn, int logbeta,
                const Tables& T, hipStream_t s);
// entries of the four-step table for (logn, logbeta) (inverse: logbeta = -1), and its generator
u64 fourstep_size(int logn, int logbeta);
void build_fourstep(u64* out, int logn, int logbeta, const Tables& T, hipStream_t s);
// the pass tables alone (forward, for sizes without a four-step table): entries and generator
u64 pass_tables_size(int logn, int logbeta);
void build_pass_tables(u64* out, int logn, int logbeta, const Tables& T, hipStream_t s);
// field-primitive self test (xfg_debug_field): op 0 mul, 1 add, 2 sub, 3 canon(a), 4 a * 2^b,
// 5 fold(a, (u32)b), 6 sub_weak(a, b), 7 add_w(a, b) (the NTT butterfly add, b < p)
void launch_field_op(int op, const u64* a, const u64* b, u64* out, u64 count, hipStream_t s);
// inverse: evals[poly][n] at 7^off7 * w_n^i -> coefficients (first `keep` written, stride out_stride)
void launch_interpolate(const u64* evals, u64 in_stride, u64* out, u64 out_stride, u64* scratch, int npoly, int logn,
                        bool off7, u64 keep, const Tables& T, hipStream_t s);

// ---- device-side Fiat-Shamir (winter-crypto DefaultRandomCoin<Blake3_256>, as host_common.hpp Coin).
// Each transcript step runs in the kernel that produces its input, one proof per block; the host
// replays the same steps from the roots and the OOD frame afterwards. fail[b] = 1 when a draw was
// rejected 1000 times in a row or z = 0.
struct DevCoin {
    Digest seed;
    u64 counter;
    u64 pad;
};
// step run on a Merkle root by launch_tree_top: reseed with the root, then
//   COEFFS (trace root): the 15 composition coefficients -> out = coeffs [B][15][D]
//   OOD_POINT (composition root): z -> out = zpts [B][2][D] = (z, z g)
//   FRI_ALPHA (FRI layer root): alpha -> out = alpha7 [B][D] = alpha * 7^-1
struct CoinStep {
    enum Kind : int { NONE = 0, COEFFS = 1, OOD_POINT = 2, FRI_ALPHA = 3 };
    int kind = NONE;
    int ext = 1;
    DevCoin* coins = nullptr;
    int* fail = nullptr;
    u64* out = nullptr;
    u64 g = 0;                  // OOD_POINT: the trace domain generator
    Digest* root_out = nullptr;  // root of proof b also stored at root_out[b] (one contiguous D2H)
    u64* hist = nullptr;         // FRI_ALPHA: the raw alpha of proof b also stored at hist[b][D]
};
// step run by launch_ood on the OOD frame (when coins is set): reseed with hash(trace frame) and
// hash(H(z)), draw a_0..a_6 and gamma, and form the DEEP parameters dp [B] from zpts [B][2][D]
struct DeepCoinStep {
    DevCoin* coins = nullptr;
    int* fail = nullptr;
    const u64* zpts = nullptr;
    DeepParams* dp = nullptr;
    u64 ginv = 0;  // g^-1
};

// self test of the draw paths (xfg_debug_coin_draws): from coin c0, k <= 64 draws by one wave
// (out_wave) and one at a time (out_seq), both [k][2]; counters after each in ctr[2], success in ok[2]
void launch_coin_draw_test(const DevCoin& c0, int k, int ext, const u64* rej, u64* out_wave, u64* out_seq, u64* ctr,
                           int* ok, hipStream_t s);

// ---- Merkle (heap layout: nodes[1] = root, nodes[L + i] = leaf i) ----
// LDE commitments store levels >= log2(beta) + 1 only: node_stride >= 2n; the subtree over rows
// (2j, 2j+1) tops out at heap node n/2 + j; launch_tree_top(nodes, stride, n / 2, ...) finishes
// also merges each block's nodes a few levels up; returns the node count of the highest level
// written (finish with launch_tree_top(nodes, stride, returned count, ...))
u64 launch_leaves_lde(const u64* lde, int nc, Digest* nodes, u64 node_stride, int npoly, int logn, int logbeta,
                      hipStream_t s);
// recompute the local subtree heap (2 * beta digests, slot 1 = top, leaf t at beta + t) of LDE
// rows entries[e] = proof << logn | m, for Merkle openings
void launch_open_rows(const u64* lde, int nc, const u64* entries, u64 count, Digest* out, int logn, int logbeta,
                      hipStream_t s);
// FRI layer leaves: row i = values at natural indices i + k*rows, k < 8 (coset-major source when
// coset_major, else natural); all leaves stored at nodes[rows + i]
// (returns the node count left for launch_tree_top, like launch_leaves_lde)
u64 launch_fri_leaves(const u64* vals, u64 val_stride, u64 comp_stride, bool coset_major, int logn, int logbeta,
                      u64 rows, Digest* nodes, u64 node_stride, int npoly, int ext, hipStream_t s);
// completes the tree above level `count` (nodes [count, 2count) present) up to the root, then runs
// the transcript step `cs` on it
void launch_tree_top(Digest* nodes, u64 node_stride, u64 count, int npoly, hipStream_t s,
                     const CoinStep& cs = CoinStep{});

// ---- AIR ----
void launch_trace_gen(const AirConst* air, u64* trace, int logn, int npoly, hipStream_t s);
// composition evaluations over the CE domain 7*<w_2n> (natural order) from the trace LDE
// div = constraint divisor table [3][2][n] from ce_divisor_table()
// ext = extension degree D: coeffs [B][15][D], ce planes [B][D][2n]
void launch_constraint_eval(const u64* lde, const AirConst* air, const u64* coeffs, const u64* div, u64* ce, int logn,
                            int logbeta, int npoly, int ext, hipStream_t s);

// ---- OOD / DEEP ----
// partial: [B][ood_partial_count(logn)][15] per-block sums, kept for launch_deep
// ext = D: zpts [B][2][D], hcoef planes [B][D][n], partial [B][count][15][D], ood [B][15][D]
void launch_ood(const u64* coef, const u64* hcoef, const u64* zpts, u64* partial, u64* ood, int logn, int npoly,
                int ext, hipStream_t s, const DeepCoinStep& dc = DeepCoinStep{});
u64 ood_partial_count(int logn);
// carry: [B][ood_partial_count(logn)][2][D]; deep planes [B][D][n]
void launch_deep(const u64* coef, const u64* hcoef, const DeepParams* dp, const u64* partial, u64* carry, u64* deep,
                 int logn, int npoly, int ext, hipStream_t s);

// ---- FRI ----
// alpha7 [B][D] = alpha * 7^-1; E values as D planes comp_stride apart; out planes [B][D][out_stride]
void launch_fri_fold(const u64* vals, u64 val_stride, u64 comp_stride, bool coset_major, int logn, int logbeta,
                     u64 rows, int logD, const u64* alpha7, u64* out, u64 out_stride, const Tables& T, int npoly,
                     int ext, hipStream_t s);

// ---- openings ----
// several gathers in one launch: segment k copies src[k][idx[first[k] + j]] to dst[k][j],
// j < first[k + 1] - first[k], as u64 or as Digest (digest[k])
struct GatherSet {
    static constexpr int MAX = 24;
    int nseg = 0;
    const void* src[MAX];
    void* dst[MAX];
    int digest[MAX];
    u64 first[MAX + 1] = {0};
};
void launch_gather_set(const GatherSet& g, const u64* idx, hipStream_t s);

// contiguous device regions packed end to end into one block (segment k: words[k] 32-bit words
// from src[k] to dst + off[k] words); dst may be device-mapped pinned host memory
struct PackSet {
    static constexpr int MAX = 12;
    int nseg = 0;
    const void* src[MAX];
    u64 off[MAX], words[MAX];
};
void launch_pack(const PackSet& p, void* dst, hipStream_t s);

}  // namespace xfg
