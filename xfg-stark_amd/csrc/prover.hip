// Host orchestration of the MI355X burn-proof STARK prover + the C ABI (include/xfg_stark.h).
//
// Pipeline = Winterfell 0.8.3 `Prover::prove` as bound by the reference
// (src/burn_mint_air.rs:479-531, src/burn_mint_prover.rs:62-129), batched over independent
// proofs: every kernel launch covers all proofs of the batch, and the host only touches the
// serial Fiat-Shamir steps (a few BLAKE3 calls per proof per round) between launch sets.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <mutex>
#include <condition_variable>
#include <deque>
#include <vector>

#include "../../include/xfg_stark.h"
#include "host_common.hpp"
#include "host_pool.hpp"
#include "kernels.hpp"
#include "verifier.hpp"

namespace xfg {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess)                                                                      \
            throw HipError(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x);        \
    } while (0)

// ------------------------------------------------------------------ marshalling
static const u64 STANDARD_BURN = 8000000ULL, LARGE_BURN = 8000000000ULL;
static u64 le_u32(const uint8_t* b) {
    return (u64)b[0] | ((u64)b[1] << 8) | ((u64)b[2] << 16) | ((u64)b[3] << 24);
}
static u64 le_u64(const uint8_t* b) { return le_u32(b) | (le_u32(b + 4) << 32); }
static void put_le64(uint8_t* d, u64 v) {
    for (int i = 0; i < 8; i++) d[i] = (uint8_t)(v >> (8 * i));
}

// compute_nullifier / compute_recipient_hash / compute_commitment (src/burn_mint_air.rs:124-202)
static void air_constants(const u64 pub[12], u64 secret, u64& nullifier, u64& commitment) {
    uint8_t buf[160], h[32], rf[32];
    size_t k = 0;
    put_le64(buf, secret);
    k = 8;
    memcpy(buf + k, "nullifier", 9);
    k += 9;
    put_le64(buf + k, pub[0]);
    k += 8;
    keccak256(buf, k, h);
    nullifier = le_u32(h);
    k = 0;
    put_le64(buf, pub[3]);
    k = 8;
    memcpy(buf + k, "ethereum-recipient", 18);
    k += 18;
    memcpy(buf + k, "fuego-to-heat-bridge", 20);
    k += 20;
    keccak256(buf, k, rf);
    k = 0;
    const u64 fields[3] = {secret, pub[0], pub[1]};
    for (u64 f : fields) { put_le64(buf + k, f); k += 8; }
    for (int i = 0; i < 4; i++) { put_le64(buf + k, pub[5 + i]); k += 8; }
    memcpy(buf + k, rf, 32);
    k += 32;
    for (int i = 0; i < 3; i++) { put_le64(buf + k, pub[9 + i]); k += 8; }
    memcpy(buf + k, "heat-commitment-v1", 18);
    k += 18;
    keccak256(buf, k, h);
    commitment = le_u32(h);
}

// validate_inputs + prove_burn_mint marshalling (src/burn_mint_prover.rs:62-118, 132-221)
static int marshal(const xfg_burn_inputs* in, AirConst& a, std::string& err) {
    u64 legacy = le_u64(in->tx_prefix_hash);
    if (in->burn_amount != STANDARD_BURN && in->burn_amount != LARGE_BURN) {
        err = "Burn amount must be exactly 0.8 XFG (8,000,000 atomic units) or 800 XFG (8,000,000,000 atomic units)";
        return XFG_INVALID_BURN_AMOUNT;
    }
    if (in->mint_amount != in->burn_amount) {
        err = "Mint amount " + std::to_string(in->mint_amount) + " does not match burn amount " +
              std::to_string(in->burn_amount) + " for 1:1 atomic unit conversion";
        return XFG_MINT_MISMATCH;
    }
    if (legacy == 0) {
        err = "Transaction hash must be greater than 0";
        return XFG_ZERO_TX_HASH;
    }
    if (!in->recipient_address || in->recipient_len != 20) {
        err = "Recipient address must be exactly 20 bytes";
        return XFG_BAD_RECIPIENT_LEN;
    }
    if (!in->secret || in->secret_len < 4) {
        err = "Secret must be at least 4 bytes";
        return XFG_SHORT_SECRET;
    }
    if (in->secret_len < 8) {  // the reference slices secret[..8] and panics (:203-204)
        err = "Secret must be at least 8 bytes (secret[..8] slice in secret_to_field_element)";
        return XFG_SHORT_SECRET;
    }
    u64 secret = le_u32(in->secret);
    uint8_t buf[29], h[32];
    memcpy(buf, in->recipient_address, 20);
    memcpy(buf + 20, "recipient", 9);
    keccak256(buf, 29, h);
    memset(&a, 0, sizeof a);
    a.pub[0] = (uint32_t)in->burn_amount;
    a.pub[1] = (uint32_t)in->mint_amount;
    a.pub[2] = (uint32_t)legacy;
    a.pub[3] = le_u32(h);
    a.pub[4] = 0;
    for (int i = 0; i < 4; i++) a.pub[5 + i] = le_u32(in->tx_prefix_hash + 4 * i);
    a.pub[9] = in->network_id;
    a.pub[10] = in->target_chain_id;
    a.pub[11] = in->commitment_version;
    air_constants(a.pub, secret, a.nullifier, a.commitment);
    return XFG_OK;
}

// ------------------------------------------------------------------ byte writer
struct BW {
    std::vector<uint8_t>& b;  // caller-owned scratch, reused across proofs (never shrunk)
    size_t o = 0;
    explicit BW(std::vector<uint8_t>& buf) : b(buf) {}
    void reserve(size_t k) {
        if (b.size() < k) b.resize(k);
    }
    uint8_t* at(size_t k) {  // k bytes at the cursor (grows geometrically; callers pre-size)
        if (o + k > b.size()) b.resize(std::max(2 * b.size(), o + k));
        uint8_t* q = b.data() + o;
        o += k;
        return q;
    }
    void put(const void* p, size_t k) { memcpy(at(k), p, k); }
    void u8(u64 v) { *at(1) = (uint8_t)v; }
    void u16(u64 v) { uint16_t x = (uint16_t)v; put(&x, 2); }  // little-endian host
    void u32(u64 v) { uint32_t x = (uint32_t)v; put(&x, 4); }
    void u64_(u64 v) { put(&v, 8); }
    void u64s(const u64* v, size_t k) { put(v, 8 * k); }
    void digest(const Digest& d) { put(d.w, 32); }  // LE words == digest bytes
    size_t len_slot() { at(4); return o; }          // u32 byte length of what follows
    void len_patch(size_t end_of_slot) {
        uint32_t x = (uint32_t)(o - end_of_slot);
        memcpy(b.data() + end_of_slot - 4, &x, 4);
    }
    void finish(std::vector<uint8_t>& out) { out.assign(b.begin(), b.begin() + o); }
    void trim() { b.resize(o); }  // the buffer is the output (the proof's own bytes)
};

// XFG_TRACE=1: host-side phase timestamps of every prove call (and any workspace reallocation,
// which synchronises the device), printed to stderr
static bool trace_on() {
    static const bool on = getenv("XFG_TRACE") && *getenv("XFG_TRACE") == '1';
    return on;
}
static void trace_realloc(const char* kind, size_t old_n, size_t new_n, size_t elem) {
    if (trace_on()) fprintf(stderr, "[xfg] realloc %s %zu -> %zu bytes\n", kind, old_n * elem, new_n * elem);
}

// ------------------------------------------------------------------ device buffers
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t cnt) {
        if (cnt <= n) return;
        trace_realloc("device", n, std::max<size_t>(cnt + cnt / 8, 1), sizeof(T));
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t want = std::max<size_t>(cnt + cnt / 8, 1);
        HIPCHK(hipMalloc((void**)&p, want * sizeof(T)));
        n = want;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// pinned host staging (hipHostMalloc) so D2H/H2D copies are true async DMA, grown with headroom.
// Flags: hipHostMallocDefault for DMA staging; MappedHBuf for the blocks kernels read and write in
// place through hipHostGetDevicePointer (the per-unit AIR constants, coins, replay block, opening
// indices / values / digests): fine-grained (coherent) memory, so a kernel never reads a line the GPU
// cached for an earlier unit and its stores reach the host without relying on the dispatch packets'
// system-scope release (coarse-grained host memory is coherent only at those fences).
template <class T, unsigned Flags = hipHostMallocDefault>
struct HBuf {
    T* p = nullptr;
    size_t n = 0;
    T* ensure(size_t cnt) {
        if (cnt <= n) return p;
        trace_realloc("pinned", n, cnt + cnt / 4 + 16, sizeof(T));
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        size_t want = cnt + cnt / 4 + 16;
        HIPCHK(hipHostMalloc((void**)&p, want * sizeof(T), Flags));
        n = want;
        return p;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    T& operator[](size_t i) { return p[i]; }
    T* data() { return p; }
};

template <class T>
using MappedHBuf = HBuf<T, hipHostMallocMapped | hipHostMallocCoherent>;

struct TablesHost {
    int LM = -1;
    DBuf<u64> tw, pow7, ipow7;
    std::map<int, DBuf<u64>> ce_div;  // constraint divisor tables per log2(trace length)
    FourStep fs;                      // four-step twiddle tables (pointers into four_buf)
    std::map<int, DBuf<u64>> four_buf;
    std::map<int, DBuf<u64>> pass_buf;  // standalone forward pass tables (fs.pass_fwd)
};

// Data-independent constraint divisors on the CE domain x_i = 7 w_2n^i (i = 2m + par), laid out
// [3][par][m]: transition (x - g^(n-1)) / (x^n - 1), boundary 1/(x - 1) and 1/(x - g^(n-1))
// (ConstraintDivisor::from_transition / from_assertion). Batch-inverted once per trace length.
static std::vector<u64> ce_divisor_table(int logn) {
    const u64 n = 1ULL << logn, nce = 2 * n;
    const u64 w = gl_root(logn + 1), g_last = gl_pow(gl_root(logn), n - 1);
    const u64 sn = gl_pow(GEN, n);
    const u64 inv_xn1[2] = {gl_inv(gl_sub(sn, 1)), gl_inv(gl_sub(gl_neg(sn), 1))};
    std::vector<u64> xa(nce), xb(nce), prod(nce);
    u64 x = GEN, acc = 1;
    for (u64 i = 0; i < nce; i++, x = gl_mul(x, w)) {
        xa[i] = gl_sub(x, 1);
        xb[i] = gl_sub(x, g_last);
        acc = gl_mul(acc, gl_mul(xa[i], xb[i]));
        prod[i] = acc;
    }
    u64 inv = gl_inv(acc);
    std::vector<u64> out(3 * nce);
    for (u64 i = nce; i-- > 0;) {
        u64 inv_ab = i ? gl_mul(inv, prod[i - 1]) : inv;  // 1 / (xa_i xb_i)
        inv = gl_mul(inv, gl_mul(xa[i], xb[i]));
        const u64 par = i & 1, m = i >> 1, di = par * n + m;
        out[di] = gl_mul(xb[i], inv_xn1[par]);
        out[nce + di] = gl_mul(inv_ab, xb[i]);
        out[2 * nce + di] = gl_mul(inv_ab, xa[i]);
    }
    return out;
}

static const char* STAGE_NAMES[] = {"trace_lde",     "trace_commit", "constraint_eval", "composition",
                                    "comp_commit",   "ood",          "deep",            "fri",
                                    "queries_gather", "host_total",  "host_queries",    "host_serialize"};
enum {
    ST_LDE, ST_TCOMMIT, ST_CE, ST_COMP, ST_CCOMMIT, ST_OOD, ST_DEEP, ST_FRI, ST_GATHER, ST_HOST, ST_HQUERY, ST_HSER,
    ST_COUNT
};

// one proof's opening plan (prove_lane step 7): the batch openings of the LDE trees and the FRI
// layers, and its gather indices per source (values: trace LDE, composition LDE, FRI layers;
// digests: trace / composition tree nodes, FRI layer nodes) and recomputed-subtree rows
struct LaneLayout {
    BatchOpening op;                     // trace / constraint trees (same positions)
    std::vector<int64_t> ref;            // per node: >= 0 stored ordinal, < 0 -(open slot + 1), slots from this proof's first
    std::vector<BatchOpening> fops;      // FRI layers
    std::vector<std::vector<u64>> fpos;
    std::vector<u64> vlde, vh, dt, dh, oent;
    std::vector<std::vector<u64>> vf, df;
};

// one lane = one HIP stream + its pooled device buffers + one host thread; a batch is split
// across lanes so one lane's host-side Fiat-Shamir / serialisation overlaps another's kernels
struct Lane {
    hipStream_t stream = nullptr;
    hipStream_t gstream = nullptr;  // the openings' gathers (gather_stream)
    bool timing = false;
    double stage_ms[ST_COUNT] = {0};
    hipEvent_t ev[ST_COUNT + 1] = {};
    // xfg_lde_probe: events around the trace LDE launch set, totals of the units so far
    bool lde_probe = false;
    hipEvent_t lde_ev[2] = {};
    double lde_ms = 0;
    u64 lde_sets = 0, lde_polys = 0;
    DBuf<AirConst> air;
    DBuf<u64> coeffs, trace, coef, scratch, lde, ce, hcoef, hlde, zpts, partial, ood, carry, deep, f0, alpha7,
        rem, dn2, falpha;
    DBuf<Digest> tnodes, hnodes, droots;
    DBuf<DeepParams> dp;
    DBuf<DevCoin> dcoin;  // device-side transcript
    DBuf<int> dfail;
    std::vector<DBuf<u64>> flayer;
    std::vector<DBuf<Digest>> fnodes;
    // pinned host staging
    MappedHBuf<Digest> h_gd;
    MappedHBuf<u64> h_idx, h_gv;
    MappedHBuf<unsigned char> h_xfer;  // the replay's inputs, written by launch_pack
    MappedHBuf<AirConst> h_air;
    MappedHBuf<DevCoin> h_coin;
    // host scratch of the opening plans and the serialiser, kept across units so steady-state
    // units neither allocate nor page-fault (their cost grew with the shared hosts' load)
    struct {
        std::vector<u64> allidx;
        std::vector<LaneLayout> lay;
    } hs;
    void release() {
        h_gd.release();
        for (auto* b : {&h_idx, &h_gv}) b->release();
        h_xfer.release();
        h_air.release();
        h_coin.release();
        dcoin.release();
        dfail.release();
        air.release();
        for (auto* b : {&coeffs, &trace, &coef, &scratch, &lde, &ce, &hcoef, &hlde, &zpts, &partial, &ood,
                        &carry, &deep, &f0, &alpha7, &rem, &dn2, &falpha})
            b->release();
        for (auto* b : {&tnodes, &hnodes, &droots}) b->release();
        dp.release();
        for (auto& b : flayer) b.release();
        for (auto& b : fnodes) b.release();
    }
};

}  // namespace xfg

namespace xfg {
struct Batch;
struct Unit {
    Batch* b;
    int b0, b1;
    int lane;  // -1: any worker
};
}  // namespace xfg

struct xfg_ctx {
    int device = 0;
    std::string err;
    bool timing = false;
    bool lde_probe = false;  // xfg_lde_probe state, inherited by lanes created later
    xfg::TablesHost tables;
    std::vector<std::unique_ptr<xfg::Lane>> lanes;
    // persistent lane workers: one host thread per lane pulls proof units from a FIFO shared by
    // every submitted batch, so the host tail of one batch overlaps the kernels of the next
    std::mutex qm;
    std::condition_variable qcv, dcv;
    std::deque<xfg::Unit> q;
    std::vector<std::thread> workers;
    bool stop = false;
    uint64_t next_ticket = 1;
    std::map<uint64_t, std::unique_ptr<xfg::Batch>> pending;
    int last_lane = 0;
    int idle = 0;  // lane workers waiting for a unit
    // batched GPU verification workspace (xfg_verify_batch_gpu)
    struct {
        xfg::HBuf<uint8_t> stage;  // pinned: proof blob + task lists, one DMA
        xfg::DBuf<uint8_t> dstage;
        xfg::DBuf<uint32_t> flags;
        std::vector<xfg::VState> st;        // per-proof transcript states, reused between calls
        std::vector<xfg::VerifyPlan> frag;  // per-proof plan fragments, reused between calls
    } vb;
};

namespace xfg {

static void ensure_tables(xfg_ctx* c, int LM) {
    if (c->tables.LM >= LM) return;
    u64 M = 1ULL << LM;
    std::vector<u64> tw(M), p7(M), ip7(M);
    u64 w = gl_root(LM), x = 1, y = 1, z = 1, i7 = gl_inv(GEN);
    for (u64 e = 0; e < M; e++) {
        tw[e] = x;
        p7[e] = y;
        ip7[e] = z;
        x = gl_mul(x, w);
        y = gl_mul(y, GEN);
        z = gl_mul(z, i7);
    }
    c->tables.tw.release();
    c->tables.pow7.release();
    c->tables.ipow7.release();
    c->tables.tw.ensure(M);
    c->tables.pow7.ensure(M);
    c->tables.ipow7.ensure(M);
    HIPCHK(hipMemcpy(c->tables.tw.p, tw.data(), M * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->tables.pow7.p, p7.data(), M * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->tables.ipow7.p, ip7.data(), M * 8, hipMemcpyHostToDevice));
    c->tables.LM = LM;
}
static const u64* ensure_ce_table(xfg_ctx* c, int logn) {
    auto& d = c->tables.ce_div[logn];
    if (!d.p) {
        std::vector<u64> t = ce_divisor_table(logn);
        d.ensure(t.size());
        HIPCHK(hipMemcpy(d.p, t.data(), t.size() * 8, hipMemcpyHostToDevice));
    }
    return d.p;
}
static Tables tables_of(xfg_ctx* c) {
    Tables T;
    T.tw = c->tables.tw.p;
    T.LM = c->tables.LM;
    T.pow7 = c->tables.pow7.p;
    T.ipow7 = c->tables.ipow7.p;
    T.fs = &c->tables.fs;
    return T;
}
// four-step twiddle tables of the NTT sizes one (n, beta) proof uses: the forward LDE and the
// inverse NTTs of sizes 8 .. 2n (trace, composition, FRI remainder). Sizes whose table would exceed
// 2^FOURSTEP_MAX_LOG entries get the per-size pass tables instead (at 2^20 with the n-entry [k1][j2]
// table of ntt_pass_a_r1024: a full 2^24-entry table for configs[4] measured slower).
// Returns false when one is missing.
// largest log2(n beta) with a forward four-step table
static int fwd_table_max_log() { return FOURSTEP_MAX_LOG; }
static bool fourstep_ready(xfg_ctx* c, int logn, int logbeta) {
    const FourStep& f = c->tables.fs;
    if (logn + logbeta <= fwd_table_max_log() && !f.fwd[logn][logbeta]) return false;
    if (logn + logbeta > fwd_table_max_log() && logn <= PASS_MAX_LOG && !f.pass_fwd[logn][logbeta]) return false;
    for (int l = 3; l <= std::min(logn + 1, FOURSTEP_MAX_LOG); l++)
        if (!f.inv[l]) return false;
    return true;
}
// caller guarantees no kernel in flight reads the registry (fresh context or drained)
static void ensure_fourstep(xfg_ctx* c, int logn, int logbeta) {
    if (fourstep_ready(c, logn, logbeta)) return;
    ensure_tables(c, std::max(logn + logbeta, logn + 1));
    const Tables T = tables_of(c);
    auto build = [&](int ln, int lb) {
        DBuf<u64>& b = c->tables.four_buf[ln * 8 + lb + 1];
        b.ensure(fourstep_size(ln, lb));
        build_fourstep(b.p, ln, lb, T, 0);
        return (const u64*)b.p;
    };
    FourStep& f = c->tables.fs;
    if (logn + logbeta <= fwd_table_max_log() && !f.fwd[logn][logbeta]) f.fwd[logn][logbeta] = build(logn, logbeta);
    if (logn + logbeta > fwd_table_max_log() && logn <= PASS_MAX_LOG && !f.pass_fwd[logn][logbeta]) {
        DBuf<u64>& b = c->tables.pass_buf[logn * 8 + logbeta];
        b.ensure(pass_tables_size(logn, logbeta));
        build_pass_tables(b.p, logn, logbeta, T, 0);
        f.pass_fwd[logn][logbeta] = b.p;
    }
    for (int l = 3; l <= std::min(logn + 1, FOURSTEP_MAX_LOG); l++)
        if (!f.inv[l]) f.inv[l] = build(l, -1);
    HIPCHK(hipStreamSynchronize(0));
}

struct ProofJob {
    AirConst air;
    Coin coin;
    std::vector<uint8_t> commitments;
    u64 ood[30];           // 15 E elements ([T_c(z), T_c(zg)] x 7, H(z)), DE coordinates each
    std::vector<u64> rem;  // FRI remainder, E elements
    u64 nonce = 0;
    std::vector<u64> pos;
    std::vector<uint8_t> bytes;
    int status = XFG_OK;
};

static void stage_mark(Lane* c, int k, hipStream_t on = nullptr) {
    if (c->timing) HIPCHK(hipEventRecord(c->ev[k], on ? on : c->stream));
}
struct HostTrace {
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> m;
    std::map<std::string, double> acc;  // accumulated sub-phase ms
    using clk = std::chrono::steady_clock;
    clk::time_point t_ = {};
    void tic() {
        if (trace_on()) t_ = clk::now();
    }
    void toc(const char* what) {
        if (!trace_on()) return;
        auto t = clk::now();
        acc[what] += std::chrono::duration<double, std::milli>(t - t_).count();
        t_ = t;
    }
    void mark(const char* what) {
        if (trace_on()) m.push_back({what, std::chrono::steady_clock::now()});
    }
    void dump(int B) {
        if (!trace_on() || m.size() < 2) return;
        std::string line = "[xfg] B=" + std::to_string(B);
        for (size_t i = 1; i < m.size(); i++) {
            char buf[96];
            snprintf(buf, sizeof buf, " %s=%.2f", m[i].first,
                     std::chrono::duration<double, std::milli>(m[i].second - m[i - 1].second).count());
            line += buf;
        }
        for (auto& kv : acc) {
            char buf[96];
            snprintf(buf, sizeof buf, " [%s=%.3f]", kv.first.c_str(), kv.second);
            line += buf;
        }
        fprintf(stderr, "%s\n", line.c_str());
    }
};

// the lane's stream for the openings' gathers, at the highest stream priority (a second stream at
// the default priority measured 4-5 % slower)
// created when the lanes are (ensure_lanes, after every lane's proving stream): a high-priority stream
// costs ~10 ms to create, which a lazily created one added to the first unit every lane ran (XFG_TRACE,
// profiles/r06/host_phases.txt); lane 0 used alone (the debug / bench entry points) creates it here
static hipStream_t gather_stream(Lane* c) {
    if (!c->gstream) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
        HIPCHK(hipStreamCreateWithPriority(&c->gstream, hipStreamNonBlocking, greatest));
    }
    return c->gstream;
}

// the batched prover: jobs[i].air filled; trace_host optional ([B][7][n], else generated on device)
static void prove_lane(Lane* c, const Tables& T, const u64* ce_div, ProofJob* jobs_p, int B, const u64* trace_host,
                       u64 n, const Opts& o) {
    auto t_host0 = std::chrono::steady_clock::now();
    HostTrace ht;
    ht.mark("start");
    struct JobSpan {
        ProofJob* p;
        int k;
        ProofJob& operator[](int i) { return p[i]; }
        ProofJob* begin() { return p; }
        ProofJob* end() { return p + k; }
    } jobs{jobs_p, B};
    const int logn = (int)ilog2(n), logbeta = (int)ilog2(o.beta);
    const u64 beta = o.beta, N = n * beta;
    const unsigned nl = num_fri_layers(N, o);
    const int DE = (int)o.ext;  // extension degree: E-valued data is DE coordinate planes
    hipStream_t s = c->stream;

    // ---- buffers
    c->air.ensure(B);
    c->coeffs.ensure((size_t)B * 15 * DE);
    c->trace.ensure((size_t)B * 7 * n);
    c->coef.ensure((size_t)B * 7 * n);
    c->scratch.ensure((size_t)B * 7 * N);
    c->lde.ensure((size_t)B * 7 * N);
    c->tnodes.ensure((size_t)B * 2 * n);
    c->ce.ensure((size_t)B * DE * 2 * n);
    c->hcoef.ensure((size_t)B * DE * n);
    c->hlde.ensure((size_t)B * DE * N);
    c->hnodes.ensure((size_t)B * 2 * n);
    c->zpts.ensure((size_t)B * 2 * DE);
    c->partial.ensure((size_t)B * 15 * DE * ood_partial_count(logn));
    c->ood.ensure((size_t)B * 15 * DE);
    c->dp.ensure(B);
    c->carry.ensure((size_t)B * 2 * DE * ood_partial_count(logn));
    c->deep.ensure((size_t)B * DE * n);
    c->f0.ensure((size_t)B * DE * N);
    c->alpha7.ensure((size_t)B * DE);
    c->falpha.ensure((size_t)std::max(1u, nl) * B * DE);
    c->dn2.ensure((size_t)B * DE);
    if (c->flayer.size() < nl + 1) {
        c->flayer.resize(nl + 1);
        c->fnodes.resize(nl + 1);
    }
    std::vector<u64> D(nl + 1);
    D[0] = N;
    for (unsigned l = 1; l <= nl; l++) D[l] = D[l - 1] / o.fold;
    for (unsigned l = 0; l < nl; l++) {
        c->fnodes[l].ensure((size_t)B * 2 * (D[l] / o.fold));
        c->flayer[l + 1].ensure((size_t)B * DE * D[l + 1]);
    }
    const u64 rem_len = N >> (3 * nl) >> logbeta;  // D_final / blowup
    c->rem.ensure((size_t)B * DE * std::max<u64>(rem_len, 1));
    {
        // opening buffers (pinned, device-mapped: the gathers read and write them directly) sized by
        // upper bounds once, so steady-state calls never re-allocate (hipHostMalloc would serialise
        // the device and the other lanes)
        const size_t q = o.q, depth = logn + logbeta;
        const size_t vals = (size_t)B * q * (7 + DE + 8 * DE * nl);
        size_t digs = (size_t)B * q * 2 * depth;
        for (unsigned l = 0; l < nl; l++) digs += (size_t)B * q * ilog2(D[l] / 8);
        const size_t opens = (size_t)B * q * 2 * 2 * 2 * beta;
        c->h_idx.ensure(vals + digs + (size_t)B * 2 * q);
        c->h_gv.ensure(vals);
        c->h_gd.ensure(digs + opens);
    }

    // the unit's small uploads are copied by a kernel from the pinned, device-mapped host blocks: no
    // copy-engine transfer for the lane stream to wait on (see the replay's pack below). The lane
    // rewrites these blocks only for its next unit, after this one's stream has drained.
    auto upload = [&](void* dst, const void* host, size_t bytes) {
        void* hd = nullptr;
        HIPCHK(hipHostGetDevicePointer(&hd, const_cast<void*>(host), 0));
        PackSet u;
        u.src[0] = hd;
        u.off[0] = 0;
        u.words[0] = bytes / 4;
        u.nseg = 1;
        launch_pack(u, dst, s);
    };
    static_assert(sizeof(AirConst) % 4 == 0 && sizeof(DevCoin) % 4 == 0, "uploads copy 32-bit words");
    AirConst* airs = c->h_air.ensure(B);
    for (int b = 0; b < B; b++) airs[b] = jobs[b].air;
    upload(c->air.p, airs, B * sizeof(AirConst));
    // transcript seed: Context::to_elements || public inputs (ProverChannel::new)
    for (auto& j : jobs) {
        u64 e[20];
        context_elements(n, o, e);
        memcpy(e + 8, j.air.pub, 12 * 8);
        j.coin.init(e, 20);
        j.commitments.clear();
    }
    // The Fiat-Shamir steps between the commitments (coefficient, OOD point, DEEP and FRI alpha
    // draws) run on the device from a copy of each proof's coin, so the whole chain from the trace
    // to the FRI remainder is enqueued without a host round trip; the host replays the same
    // transcript from the roots and OOD values once the chain has finished (below).
    {
        DevCoin* hc = c->h_coin.ensure(B);
        for (int b = 0; b < B; b++) {
            hc[b].seed = jobs[b].coin.seed;
            hc[b].counter = jobs[b].coin.counter;
            hc[b].pad = 0;
        }
        c->dcoin.ensure(B);
        c->dfail.ensure(B);
        upload(c->dcoin.p, hc, B * sizeof(DevCoin));
        HIPCHK(hipMemsetAsync(c->dfail.p, 0, B * sizeof(int), s));
    }

    // ---- 1. trace LDE + commitment (DefaultTraceLde::new)
    ht.mark("setup");
    stage_mark(c, 0);
    if (trace_host) HIPCHK(hipMemcpyAsync(c->trace.p, trace_host, (size_t)B * 7 * n * 8, hipMemcpyHostToDevice, s));
    else launch_trace_gen(c->air.p, c->trace.p, logn, B, s);
    launch_interpolate(c->trace.p, n, c->coef.p, n, c->scratch.p, B * 7, logn, false, n, T, s);
    const bool probe = c->lde_probe;
    if (probe) {
        if (!c->lde_ev[0]) {
            HIPCHK(hipEventCreate(&c->lde_ev[0]));
            HIPCHK(hipEventCreate(&c->lde_ev[1]));
        }
        HIPCHK(hipEventRecord(c->lde_ev[0], s));
    }
    launch_lde(c->coef.p, n, c->lde.p, c->scratch.p, B * 7, logn, logbeta, T, s);
    if (probe) HIPCHK(hipEventRecord(c->lde_ev[1], s));
    stage_mark(c, 1);
    // ---- 2. trace root -> constraint composition coefficients (7 transition + 8 boundary)
    CoinStep cs;
    cs.ext = DE;
    cs.coins = c->dcoin.p;
    cs.fail = c->dfail.p;
    c->droots.ensure((size_t)(2 + nl) * B);  // trace, composition, FRI layer roots: [tree][B]
    cs.kind = CoinStep::COEFFS;
    cs.out = c->coeffs.p;
    cs.root_out = c->droots.p;
    launch_tree_top(c->tnodes.p, 2 * n, launch_leaves_lde(c->lde.p, 7, c->tnodes.p, 2 * n, B, logn, logbeta, s), B,
                    s, cs);
    stage_mark(c, 2);

    // ---- 3. constraint evaluation + composition polynomial + commitment
    launch_constraint_eval(c->lde.p, c->air.p, c->coeffs.p, ce_div, c->ce.p, logn, logbeta, B, DE, s);
    stage_mark(c, 3);
    launch_interpolate(c->ce.p, 2 * n, c->hcoef.p, n, c->scratch.p, B * DE, logn + 1, true, n, T, s);
    launch_lde(c->hcoef.p, n, c->hlde.p, c->scratch.p, B * DE, logn, logbeta, T, s);
    stage_mark(c, 4);
    // ---- 4. composition root -> OOD point (z, z g); the frame, then the DEEP draws
    cs.kind = CoinStep::OOD_POINT;
    cs.out = c->zpts.p;
    cs.root_out = c->droots.p + B;
    cs.g = gl_root(logn);
    launch_tree_top(c->hnodes.p, 2 * n, launch_leaves_lde(c->hlde.p, DE, c->hnodes.p, 2 * n, B, logn, logbeta, s), B,
                    s, cs);
    stage_mark(c, 5);
    DeepCoinStep dc;
    dc.coins = c->dcoin.p;
    dc.fail = c->dfail.p;
    dc.zpts = c->zpts.p;
    dc.dp = c->dp.p;
    dc.ginv = gl_inv(cs.g);
    launch_ood(c->coef.p, c->hcoef.p, c->zpts.p, c->partial.p, c->ood.p, logn, B, DE, s, dc);
    stage_mark(c, 6);

    // ---- 5. DEEP composition polynomial (coefficient form) + its LDE
    launch_deep(c->coef.p, c->hcoef.p, c->dp.p, c->partial.p, c->carry.p, c->deep.p, logn, B, DE, s);
    launch_lde(c->deep.p, n, c->f0.p, c->scratch.p, B * DE, logn, logbeta, T, s);
    // degree check: deg(DEEP) == n - 2  <=>  coefficient n-2 != 0 (coefficient n-1 is 0 by construction)
    HIPCHK(hipMemcpy2DAsync(c->dn2.p, 8, c->deep.p + (n - 2), n * 8, 8, (size_t)B * DE, hipMemcpyDeviceToDevice, s));
    stage_mark(c, 7);

    // ---- 6. FRI layers (FriProver::build_layers), folding factor 8: commit -> reseed -> draw alpha
    // -> fold, every round on the device
    for (unsigned l = 0; l < nl; l++) {
        const u64 rows = D[l] / 8;
        const bool cm = (l == 0);
        const u64* src = cm ? c->f0.p : c->flayer[l].p;
        const u64 cstride = cm ? N : D[l], sstride = DE * cstride;
        u64 top = launch_fri_leaves(src, sstride, cstride, cm, logn, logbeta, rows, c->fnodes[l].p, 2 * rows, B, DE,
                                    s);
        cs.kind = CoinStep::FRI_ALPHA;
        cs.out = c->alpha7.p;
        cs.hist = c->falpha.p + (size_t)l * B * DE;  // the raw alpha of this layer, for the replay
        cs.root_out = c->droots.p + (size_t)(2 + l) * B;
        launch_tree_top(c->fnodes[l].p, 2 * rows, top, B, s, cs);
        launch_fri_fold(src, sstride, cstride, cm, logn, logbeta, rows, (int)ilog2(D[l]), c->alpha7.p,
                        c->flayer[l + 1].p, rows, T, B, DE, s);
    }
    ht.mark("chain_launch");
    // remainder: interpolate the last layer over 7*<w_D>, keep D/blowup coefficients
    // (with no folding layer this is the DEEP polynomial's own coefficients), planes [b][c][rem_len]
    if (nl > 0) {
        launch_interpolate(c->flayer[nl].p, D[nl], c->rem.p, rem_len, c->scratch.p, B * DE, (int)ilog2(D[nl]), true,
                           rem_len, T, s);
    } else {
        HIPCHK(hipMemcpy2DAsync(c->rem.p, rem_len * 8, c->deep.p, n * 8, rem_len * 8, (size_t)B * DE,
                                hipMemcpyDeviceToDevice, s));
    }
    // transcript inputs for the host replay (trace / composition / FRI roots, OOD frame, the device's
    // draws, DEEP parameters, FRI alphas, rejections, remainder, DEEP degree check): one kernel packs
    // them straight into the pinned host block (device-mapped, written with plain vector stores),
    // visible to the host after the stream synchronisation below. As eight hipMemcpyAsync blits each
    // could start ~0.2 ms after the previous one (rocprof, scripts/fri_timeline.sh: 1.7 ms of idle
    // stream after the last FRI fold); as one larger copy the runtime takes the SDMA engine, whose
    // dependency on the lane stream cost 17 % of the pipelined throughput (same box, lib_ab.sh)
    PackSet pk;
    u64 words = 0;
    auto seg = [&](const void* src, size_t bytes) {
        const u64 at = words;
        pk.src[pk.nseg] = src;
        pk.off[pk.nseg] = at;
        pk.words[pk.nseg++] = bytes / 4;
        words = (at + bytes / 4 + 63) & ~63ULL;  // 256 B aligned segments
        return at * 4;
    };
    const u64 o_roots = seg(c->droots.p, (size_t)(2 + nl) * B * sizeof(Digest));  // [trace, comp, FRI 0..nl-1][B]
    const u64 o_ood = seg(c->ood.p, (size_t)B * 15 * DE * 8);
    const u64 o_co = seg(c->coeffs.p, (size_t)B * 15 * DE * 8);
    const u64 o_dp = seg(c->dp.p, (size_t)B * sizeof(DeepParams));
    const u64 o_falpha = seg(c->falpha.p, (size_t)nl * B * DE * 8);  // [layer][B][DE]
    const u64 o_fail = seg(c->dfail.p, (size_t)B * sizeof(int));
    const u64 o_rem = seg(c->rem.p, (size_t)B * DE * rem_len * 8);
    const u64 o_dn2 = seg(c->dn2.p, (size_t)B * DE * 8);
    unsigned char* hx = c->h_xfer.ensure(words * 4);
    void* hx_dev = nullptr;
    HIPCHK(hipHostGetDevicePointer(&hx_dev, hx, 0));
    launch_pack(pk, hx_dev, s);
    const Digest* roots = (const Digest*)(hx + o_roots);
    const u64* ood = (const u64*)(hx + o_ood);
    const u64* co = (const u64*)(hx + o_co);
    const DeepParams* dps = (const DeepParams*)(hx + o_dp);
    const Digest* froots = roots + 2 * B;
    const u64* falpha = (const u64*)(hx + o_falpha);
    const int* ffail = (const int*)(hx + o_fail);
    const u64* remh = (const u64*)(hx + o_rem);
    const u64* dn2h = (const u64*)(hx + o_dn2);
    stage_mark(c, 8);
    ht.mark("launch_rem");
    HIPCHK(hipStreamSynchronize(s));
    ht.mark("sync_rem");
    // host replay of the transcript: commitments into the proof and the coin advanced exactly as the
    // device coin was; the device's coefficient, z and DEEP draws (and its rejections) must agree
    // (per proof, independent: spread over the host pool)
    HostPool& pool = host_pool();
    pool.parallel_for(B, [&](int b) {
        auto& j = jobs[b];
        bool failed = false, same = true;
        auto commit = [&](const Digest& r) {
            uint8_t rb[32];
            digest_bytes(r, rb);
            j.commitments.insert(j.commitments.end(), rb, rb + 32);
            j.coin.reseed(r);
        };
        auto draw = [&](const u64* dev) {  // dev: the device's value (DE coordinates) or null
            u64 a[2] = {0, 0};
            if (!j.coin.draw_e(a, DE)) failed = true;
            for (int d = 0; dev && d < DE; d++) same &= a[d] == dev[d];
            return a[0] | a[1];
        };
        const DeepParams& P = dps[b];
        commit(roots[b]);
        for (int k = 0; k < 15; k++) draw(co + ((size_t)b * 15 + k) * DE);  // composition coefficients
        commit(roots[B + b]);
        if (draw(P.z) == 0) failed = true;  // z = 0: no DEEP quotient
        memcpy(j.ood, &ood[(size_t)b * 15 * DE], 15 * DE * 8);  // [15][DE]
        j.coin.reseed(hash_elements(j.ood, 14 * DE));  // interleaved T_i(z), T_i(zg), E elements
        j.coin.reseed(hash_elements(j.ood + 14 * DE, DE));
        for (int k = 0; k < 7; k++) draw(P.a[k]);
        draw(P.gamma);
        for (unsigned l = 0; l < nl; l++) {
            commit(froots[(size_t)l * B + b]);
            draw(falpha + ((size_t)l * B + b) * DE);  // FRI alpha (the fold used alpha * 7^-1 of it)
        }
        // the DEEP parameters the device derived from z and the frame: z g, 1 / z, 1 / (z g), and the
        // OOD sums c1 = gamma H(z) + sum a_k T_k(z), c2 = sum a_k T_k(z g)
        if (!failed) {
            auto e = [&](const u64* v) { return E2{v[0], DE == 2 ? v[1] : 0}; };
            auto ood_e = [&](int q) { return E2{j.ood[q * DE], DE == 2 ? j.ood[q * DE + 1] : 0}; };
            const E2 z = e(P.z), zg = e(P.zg), one = e2(1);
            E2 c1 = e2_mul(e(P.gamma), ood_e(14)), c2{0, 0};
            for (int k = 0; k < 7; k++) {
                c1 = e2_add(c1, e2_mul(e(P.a[k]), ood_e(2 * k)));
                c2 = e2_add(c2, e2_mul(e(P.a[k]), ood_e(2 * k + 1)));
            }
            same &= e2_eq(zg, e2_mulb(z, cs.g)) && e2_eq(e2_mul(z, e(P.zinv)), one) &&
                    e2_eq(e2_mul(zg, e(P.zginv)), one) && e2_eq(c1, e(P.c1)) && e2_eq(c2, e(P.c2));
        }
        if (failed) j.status = XFG_PROVER_ERROR;
        if (failed != (ffail[b] != 0) || !same) throw std::runtime_error("device / host transcript diverged");
    });

    auto t_q0 = std::chrono::steady_clock::now();
    // ---- 7. grinding + query positions, gather lists
    // LDE trees store heap levels >= log2(beta) (indices < 2n); lower nodes of an opened row are
    // recomputed by launch_open_rows (local heap: 2 * beta slots per row). Every proof's plan is
    // built on its own (host pool) into per-proof index lists, which are then laid end to end.
    const u64 stored_lim = n, LB = beta;  // stored: heap levels >= log2(beta) + 1
    using Layout = LaneLayout;
    std::vector<Layout>& lay = c->hs.lay;
    if (lay.size() < (size_t)B) lay.resize(B);
    pool.parallel_for(B, [&](int b) {
        auto& j = jobs[b];
        Layout& L = lay[b];
        L.ref.clear();
        L.fops.clear();
        L.fpos.clear();
        for (auto* v : {&L.vlde, &L.vh, &L.dt, &L.dh, &L.oent}) v->clear();
        L.vf.resize(nl);
        L.df.resize(nl);
        if (dn2h[(size_t)b * DE] == 0 && dn2h[(size_t)b * DE + DE - 1] == 0)
            j.status = XFG_PROVER_ERROR;  // assert_eq!(trace_length - 2, degree)
        j.rem.resize(rem_len * DE);  // E elements, coordinates interleaved
        for (u64 i = 0; i < rem_len; i++)
            for (int k = 0; k < DE; k++) j.rem[i * DE + k] = remh[((size_t)b * DE + k) * rem_len + i];
        Digest rc = hash_elements(j.rem.data(), rem_len * DE);
        uint8_t rb[32];
        digest_bytes(rc, rb);
        j.commitments.insert(j.commitments.end(), rb, rb + 32);
        j.coin.reseed(rc);
        u64 nonce = 1;
        while (tz64([&] { Digest h = merge_with_int(j.coin.seed, nonce); return (u64)h.w[0] | ((u64)h.w[1] << 32); }()) <
               o.grind)
            nonce++;
        j.nonce = nonce;
        j.coin.reseed_int(nonce);
        std::vector<u64> pos(o.q);
        for (u64 i = 0; i < o.q; i++) {
            Digest h = j.coin.next();
            pos[i] = ((u64)h.w[0] | ((u64)h.w[1] << 32)) & (N - 1);
        }
        std::sort(pos.begin(), pos.end());
        pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
        j.pos = pos;
        for (u64 k : pos) {
            u64 t = k & (beta - 1), m = k >> logbeta;
            for (int col = 0; col < 7; col++) L.vlde.push_back((((u64)b * 7 + col) * beta + t) * n + m);
            for (int k = 0; k < DE; k++) L.vh.push_back((((u64)b * DE + k) * beta + t) * n + m);
        }
        // rows whose subtrees are recomputed: every queried row and its sibling row (the sibling's
        // subtree top, heap level log2(beta), is no longer stored)
        std::vector<u64> rows_b;
        for (u64 k : pos) {
            rows_b.push_back(k >> logbeta);
            rows_b.push_back((k >> logbeta) ^ 1);
        }
        std::sort(rows_b.begin(), rows_b.end());
        rows_b.erase(std::unique(rows_b.begin(), rows_b.end()), rows_b.end());
        for (u64 m : rows_b) L.oent.push_back(((u64)b << logn) | m);
        plan_batch_opening(pos, N, L.op);
        int64_t stored_ord = 0;
        L.op.each([&](u64 h) {
                if (h < stored_lim) {
                    L.dt.push_back((u64)b * 2 * n + h);
                    L.dh.push_back((u64)b * 2 * n + h);
                    L.ref.push_back(stored_ord++);
                } else {
                    // open slot relative to this proof's first entry (rebased once the entries of
                    // the proofs before it are counted)
                    unsigned lvl = (unsigned)(logn + logbeta) - (63 - __builtin_clzll(h));  // 0 = leaves
                    u64 off = h - (N >> lvl), span = logbeta - lvl;
                    u64 m = off >> span, local = (1ULL << span) + (off & ((1ULL << span) - 1));
                    u64 e = (u64)(std::lower_bound(rows_b.begin(), rows_b.end(), m) - rows_b.begin());
                    L.ref.push_back(-(int64_t)(e * 2 * LB + local) - 1);
                }
            });
        std::vector<u64> fp = pos;
        for (unsigned l = 0; l < nl; l++) {
            u64 rows = D[l] / 8;
            fp = fold_positions(fp, rows);
            L.fpos.push_back(fp);
            auto& vf = L.vf[l];
            vf.clear();
            for (u64 i : fp)
                for (u64 k = 0; k < 8; k++) {
                    const u64 K = i + k * rows;
                    for (int cc = 0; cc < DE; cc++) {
                        if (l == 0)
                            vf.push_back((((u64)b * DE + cc) * beta + (K & (beta - 1))) * n + (K >> logbeta));
                        else
                            vf.push_back(((u64)b * DE + cc) * D[l] + K);
                    }
                }
            L.fops.emplace_back();
            plan_batch_opening(fp, rows, L.fops.back());
            auto& df = L.df[l];
            df.clear();
            L.fops.back().each([&](u64 x) { df.push_back((u64)b * 2 * rows + x); });
        }
    });
    ht.mark("queries_plan");
    // one index buffer, one value buffer, one digest buffer; segment per source, the proofs' lists
    // end to end inside each segment. vcur / dcur[k * B + b]: where proof b's values / digests of segment k
    // start in the host copies gv / gd
    auto& allidx = c->hs.allidx;
    allidx.clear();
    const int NS = 2 + (int)nl;  // value segments: trace LDE, composition LDE, FRI layers (same count of digest segments)
    std::vector<std::pair<size_t, size_t>> vseg, dseg;  // (offset, count)
    std::vector<size_t> vcur((size_t)NS * B), dcur((size_t)NS * B);
    auto seg_of = [&](int k, bool dig, int b) -> const std::vector<u64>& {
        const Layout& L = lay[b];
        if (!dig) return k == 0 ? L.vlde : (k == 1 ? L.vh : L.vf[k - 2]);
        return k == 0 ? L.dt : (k == 1 ? L.dh : L.df[k - 2]);
    };
    for (int dig = 0; dig < 2; dig++)
        for (int k = 0; k < NS; k++) {
            auto& seg = dig ? dseg : vseg;
            auto& cur = dig ? dcur : vcur;
            seg.push_back({allidx.size(), 0});
            for (int b = 0; b < B; b++) {
                const auto& v = seg_of(k, dig, b);
                cur[(size_t)k * B + b] = allidx.size() - (dig ? vseg.back().first + vseg.back().second : 0);
                allidx.insert(allidx.end(), v.begin(), v.end());
            }
            seg.back().second = allidx.size() - seg.back().first;
        }
    size_t nvals = dseg.front().first;
    size_t ndig = allidx.size() - nvals;
    size_t nent = 0;
    std::vector<int64_t> ent0(B);
    for (int b = 0; b < B; b++) {
        ent0[b] = (int64_t)nent;
        allidx.insert(allidx.end(), lay[b].oent.begin(), lay[b].oent.end());
        nent += lay[b].oent.size();
    }
    const size_t nopen = nent * 2 * LB;
    u64* hidx = c->h_idx.ensure(allidx.size());
    memcpy(hidx, allidx.data(), allidx.size() * 8);
    u64* gv = c->h_gv.ensure(nvals);
    Digest* gd = c->h_gd.ensure(ndig + 2 * nopen);
    // the gathers read the indices from, and write the opened values and digests into, the pinned
    // host blocks directly (device-mapped): no copy-engine transfers whose completion the stream
    // would wait on (one larger D2H on the SDMA engine cost 17 % of the pipelined throughput, above)
    void *didx = nullptr, *dgv = nullptr, *dgd = nullptr;
    HIPCHK(hipHostGetDevicePointer(&didx, hidx, 0));
    HIPCHK(hipHostGetDevicePointer(&dgv, gv, 0));
    HIPCHK(hipHostGetDevicePointer(&dgd, gd, 0));
    const u64* gidx = (const u64*)didx;
    u64* gval = (u64*)dgv;
    Digest* gdig = (Digest*)dgd;
    ht.mark("q_idx_host");
    // the gathers (a few hundred microseconds of small kernels) go to the lane's high-priority stream:
    // on its own stream a lane's gathers queued behind the other lanes' chains in the shared hardware
    // queue (XFG_TRACE: 3.1 ms mean, 9 ms p90 to sync them); the lane's stream s has drained
    // (sync_rem), so they need no event. Timing mode takes the same stream: stage 9 is measured from
    // the lane stream's last event to an event behind the gathers' copies on this one
    const hipStream_t sq = gather_stream(c);
    ht.mark("q_h2d");
    {
        // the segments lie end to end in allidx: values first, then digests
        GatherSet gs;
        size_t vo = 0, dof = 0, gbase = 0;  // gbase: index entries consumed by launches already made
        auto add = [&](const void* src, void* dst, bool dig, size_t cnt) {
            if (gs.nseg == GatherSet::MAX) {  // very deep FRI: flush and continue in a new launch
                launch_gather_set(gs, gidx + gbase, sq);
                gbase += gs.first[gs.nseg];
                gs = GatherSet{};
            }
            gs.src[gs.nseg] = src;
            gs.dst[gs.nseg] = dst;
            gs.digest[gs.nseg] = dig ? 1 : 0;
            gs.first[gs.nseg + 1] = gs.first[gs.nseg] + cnt;
            gs.nseg++;
        };
        const u64* vsrc[2] = {c->lde.p, c->hlde.p};
        for (size_t k = 0; k < vseg.size(); k++) {
            const u64* src = k < 2 ? vsrc[k] : (k == 2 ? c->f0.p : c->flayer[k - 2].p);
            add(src, gval + vo, false, vseg[k].second);
            vo += vseg[k].second;
        }
        for (size_t k = 0; k < dseg.size(); k++) {
            const Digest* src = k == 0 ? c->tnodes.p : (k == 1 ? c->hnodes.p : c->fnodes[k - 2].p);
            add(src, gdig + dof, true, dseg[k].second);
            dof += dseg[k].second;
        }
        launch_gather_set(gs, gidx + gbase, sq);
        const u64* ent = gidx + nvals + ndig;
        launch_open_rows(c->lde.p, 7, ent, nent, gdig + ndig, logn, logbeta, sq);
        launch_open_rows(c->hlde.p, DE, ent, nent, gdig + ndig + nopen, logn, logbeta, sq);
    }
    ht.mark("q_launch");
    stage_mark(c, 9, sq);
    auto t_q1 = std::chrono::steady_clock::now();
    ht.mark("queries_host");
    HIPCHK(hipStreamSynchronize(sq));
    ht.mark("sync_gather");
    auto t_s0 = std::chrono::steady_clock::now();

    // ---- 8. StarkProof::to_bytes (DESIGN.md "Proof format"), one proof per pool task
    const Digest* open_t = gd + ndig;
    const Digest* open_h = gd + ndig + nopen;
    pool.parallel_for(B, [&](int b) {
        auto& j = jobs[b];
        const Layout& Lb = lay[b];
        const size_t eoff = (size_t)ent0[b] * 2 * LB;  // this proof's first recomputed-subtree slot
        auto write_paths = [&](BW& w, const BatchOpening& op, size_t cursor) {
            size_t slot = w.len_slot();
            w.u8(op.size());
            for (size_t i = 0; i < op.size(); i++) {
                w.u8(op.len[i]);
                w.put(&gd[cursor], 32 * op.len[i]);
                cursor += op.len[i];
            }
            w.len_patch(slot);
        };
        auto write_lde_paths = [&](BW& w, size_t cursor, const Digest* open) {
            size_t slot = w.len_slot();
            w.u8(Lb.op.size());
            size_t r = 0;
            for (size_t i = 0; i < Lb.op.size(); i++) {
                w.u8(Lb.op.len[i]);
                uint8_t* q = w.at(32 * Lb.op.len[i]);
                for (size_t k = 0; k < Lb.op.len[i]; k++, r++) {
                    int64_t ref = Lb.ref[r];
                    memcpy(q + 32 * k, (ref >= 0 ? gd[cursor++] : open[(size_t)(-ref - 1) + eoff]).w, 32);
                }
            }
            w.len_patch(slot);
        };
        const u64 nu = j.pos.size();
        BW w(j.bytes);
        w.reserve(j.commitments.size() + nu * 8 * (7 + DE + 8 * DE * nl) + (2 + nl) * nu * 32 * ilog2(N) +
                   rem_len * 8 * DE + 1024);
        // Context
        w.u8(7); w.u8(0); w.u8(logn); w.u16(0);
        w.u8(8); w.u64_(P);
        w.u8(o.q); w.u8(o.beta); w.u8(o.grind); w.u8(o.ext); w.u8(o.fold); w.u8(o.remdeg);
        w.u8(nu);
        w.u16(j.commitments.size());
        w.put(j.commitments.data(), j.commitments.size());
        // trace queries
        w.u8(1);
        w.u32(nu * 7 * 8);
        w.u64s(&gv[vcur[b]], nu * 7);
        write_lde_paths(w, dcur[b], open_t);
        // constraint queries
        w.u32(nu * 8 * DE);
        w.u64s(&gv[vcur[(size_t)B + b]], nu * DE);
        write_lde_paths(w, dcur[(size_t)B + b], open_h);
        // OOD frame (E elements)
        w.u16(1 + 14 * 8 * DE);
        w.u8(2);
        w.u64s(j.ood, 14 * DE);
        w.u16(8 * DE);
        w.u64s(j.ood + 14 * DE, DE);
        // FRI proof
        w.u8(nl);
        for (unsigned l = 0; l < nl; l++) {
            u64 nk = Lb.fpos[l].size();
            w.u32(nk * 8 * 8 * DE);
            w.u64s(&gv[vcur[(size_t)(2 + l) * B + b]], nk * 8 * DE);
            write_paths(w, Lb.fops[l], dcur[(size_t)(2 + l) * B + b]);
        }
        w.u16(rem_len * 8 * DE);
        w.u64s(j.rem.data(), rem_len * DE);
        w.u8(0);
        w.u64_(j.nonce);
        w.trim();
    });
    ht.mark("serialize");
    ht.dump(B);
    if (probe) {  // the stream has passed both events (root / query fetches synchronised it)
        float ms = 0;
        HIPCHK(hipEventSynchronize(c->lde_ev[1]));
        HIPCHK(hipEventElapsedTime(&ms, c->lde_ev[0], c->lde_ev[1]));
        c->lde_ms += ms;
        c->lde_sets++;
        c->lde_polys += (u64)B * 7;
    }
    if (c->timing) {
        for (int k = 0; k < 9; k++) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, c->ev[k], c->ev[k + 1]));
            c->stage_ms[k] = ms;
        }
        auto t_end = std::chrono::steady_clock::now();
        c->stage_ms[ST_HOST] = std::chrono::duration<double, std::milli>(t_end - t_host0).count();
        c->stage_ms[ST_HQUERY] = std::chrono::duration<double, std::milli>(t_q1 - t_q0).count();
        c->stage_ms[ST_HSER] = std::chrono::duration<double, std::milli>(t_end - t_s0).count();
    }
}

// a lane's proving stream (default priority: graded or high lane priorities measured equal or worse)
// and events
static void create_lane_stream(xfg_ctx* c, Lane* L) {
    L->lde_probe = c->lde_probe;
    HIPCHK(hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking));
    for (auto& e : L->ev) HIPCHK(hipEventCreate(&e));
}
static Lane* lane0(xfg_ctx* c) {
    if (c->lanes.empty()) {
        c->lanes.emplace_back(new Lane());
        create_lane_stream(c, c->lanes[0].get());
    }
    return c->lanes[0].get();
}
// every lane's proving stream first, then the gather streams: streams take the process's hardware
// queues (GPU_MAX_HW_QUEUES, 4) in creation order, and a gather stream created between two lanes'
// proving streams left the proving streams two of the four queues (-9 % burn-proofs/s,
// profiles/r06/gather_stream_ab.txt)
static void ensure_lanes(xfg_ctx* c, size_t k) {
    lane0(c);
    while (c->lanes.size() < k) {
        c->lanes.emplace_back(new Lane());
        create_lane_stream(c, c->lanes.back().get());
    }
    for (auto& L : c->lanes) gather_stream(L.get());
}
// lane / work-unit tuning knobs (XFG_LANES, XFG_UNIT)
static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

// ------------------------------------------------------------------ batch submission / lane workers
// a submitted batch: jobs [0, B) proven in units of XFG_UNIT proofs by the lane workers; proof
// bytes are copied into the caller's buffers on the worker thread as each unit finishes
struct Batch {
    std::vector<ProofJob> jobs;
    std::vector<uint32_t> which;   // jobs[k] -> caller index
    std::vector<uint8_t*> outs;    // caller buffers (null entry or empty: size query)
    size_t* out_lens = nullptr;    // caller capacities in, proof lengths out
    int* statuses = nullptr;       // caller statuses, written by wait
    std::vector<int> st;           // per-job copy-out status
    const u64* trace_host = nullptr;
    u64 n = 0;
    Opts o{};
    Tables T{};
    const u64* ce_div = nullptr;
    int units_left = 0;
    std::exception_ptr err;
};

static int max_lanes() {
    static const int v = std::max(1, env_int("XFG_LANES", 7));
    return v;
}
// 32 proofs per unit: a 64-proof batch is two units. Same box, 3 x 20 steps at bench.py's depth 6:
// 12,069 +- 70 burn-proofs/s against 11,890 +- 50 with 22, 11,645 with 64, 11,557 with 16. (At depth
// 3 the unit queue ran dry and smaller units won: 22 gave 11,400 against 10,790 with 32; with the
// transcript's host round trips still in place 20 had been best.)
static int unit_size() {
    static const int v = std::max(1, env_int("XFG_UNIT", 32));
    return v;
}

// smallest unit a queued unit is split into when lanes would otherwise idle (0: never split).
// 16 (a 32-proof unit splits once): with the host tail on the pool, same box, 4 interleaved 20-step
// bench runs each: 16 -> 12,725, 0 -> 12,675, 12 -> 12,576, 8 -> 12,575 burn-proofs/s (8 cut the
// first batch of a window into 8 pieces for 7 lanes)
static int split_min() {
    static const int v = std::max(0, env_int("XFG_SPLIT_MIN", 16));
    return v;
}

static void copy_unit(Batch* b, int b0, int b1) {
    host_pool().parallel_for(b1 - b0, [&](int i0) {
        const int k = b0 + i0;
        ProofJob& j = b->jobs[k];
        if (j.status) {
            b->st[k] = j.status;
            return;
        }
        if (b->which.empty()) {  // warm-up batch (xfg_prepare): bytes discarded
            std::vector<uint8_t>().swap(j.bytes);
            return;
        }
        uint32_t i = b->which[k];
        size_t need = j.bytes.size();
        uint8_t* dst = b->outs.empty() ? nullptr : b->outs[i];
        if (!dst) {
            b->st[k] = XFG_OK;  // size query (copy_out semantics)
        } else if (b->out_lens[i] >= need) {
            memcpy(dst, j.bytes.data(), need);
            b->st[k] = XFG_OK;
        } else {
            b->st[k] = XFG_BUFFER_TOO_SMALL;
        }
        b->out_lens[i] = need;
        std::vector<uint8_t>().swap(j.bytes);
    });
}

static void worker_main(xfg_ctx* c, int l) {
    (void)hipSetDevice(c->device);
    Lane* L = c->lanes[l].get();
    for (;;) {
        Unit u;
        bool skip;
        {
            std::unique_lock<std::mutex> g(c->qm);
            std::deque<Unit>::iterator it;
            auto pick = [&] {
                for (it = c->q.begin(); it != c->q.end(); ++it)
                    if (it->lane < 0 || it->lane == l) return true;
                return false;
            };
            c->idle++;
            c->qcv.wait(g, [&] { return c->stop || pick(); });
            c->idle--;
            if (c->stop) return;
            u = *it;
            c->q.erase(it);
            skip = (bool)u.b->err;  // a failed batch drops its remaining units
            L->timing = c->timing;
            // fewer queued units than idle lanes (the end of a run of batches, or a lone batch):
            // halve this unit until every idle lane has a share, the halves at the queue's front
            if (u.lane < 0 && !c->timing && !skip && split_min() > 0) {
                int avail = 0;
                for (auto& x : c->q) avail += x.lane < 0;
                bool pushed = false;
                while (u.b1 - u.b0 >= 2 * split_min() && avail < c->idle) {
                    const int mid = u.b0 + (u.b1 - u.b0) / 2;
                    c->q.push_front(Unit{u.b, mid, u.b1, -1});
                    u.b->units_left++;
                    u.b1 = mid;
                    avail++;
                    pushed = true;
                }
                if (pushed) c->qcv.notify_all();
            }
        }
        Batch* b = u.b;
        std::exception_ptr e;
        if (!skip) {
            try {
                prove_lane(L, b->T, b->ce_div, b->jobs.data() + u.b0, u.b1 - u.b0, b->trace_host, b->n, b->o);
                copy_unit(b, u.b0, u.b1);
            } catch (...) {
                e = std::current_exception();
            }
        }
        std::lock_guard<std::mutex> g(c->qm);
        if (e && !b->err) b->err = e;
        c->last_lane = l;
        if (--b->units_left == 0) c->dcv.notify_all();
    }
}

static void ensure_workers(xfg_ctx* c) {
    const int nl = max_lanes();
    ensure_lanes(c, nl);
    while ((int)c->workers.size() < nl) {
        int l = (int)c->workers.size();
        c->workers.emplace_back(worker_main, c, l);
    }
}

// blocks until no submitted unit is queued or running (tables may only be replaced then)
static void drain(xfg_ctx* c) {
    std::unique_lock<std::mutex> g(c->qm);
    c->dcv.wait(g, [&] {
        for (auto& kv : c->pending)
            if (kv.second->units_left) return false;
        return true;
    });
}

static void bind_tables(xfg_ctx* c, Batch* b) {
    const int LM = (int)(ilog2(b->n) + ilog2(b->o.beta));
    if (c->tables.LM < LM || !fourstep_ready(c, (int)ilog2(b->n), (int)ilog2(b->o.beta))) {
        drain(c);
        ensure_tables(c, LM);
        ensure_fourstep(c, (int)ilog2(b->n), (int)ilog2(b->o.beta));
    }
    b->T = tables_of(c);
    b->ce_div = ensure_ce_table(c, (int)ilog2(b->n));
}

// units of unit_size() proofs (the whole batch as one unit in timing mode, so the per-stage
// times describe one launch set of the batch)
static std::vector<Unit> split_units(xfg_ctx* c, int B) {
    std::vector<Unit> u;
    const int U = c->timing ? std::max(1, B) : unit_size();
    for (int b0 = 0; b0 < B; b0 += U) u.push_back(Unit{nullptr, b0, std::min(B, b0 + U), -1});
    return u;
}

static uint64_t enqueue(xfg_ctx* c, std::unique_ptr<Batch> bp, std::vector<Unit> units) {
    ensure_workers(c);
    Batch* b = bp.get();
    b->st.assign(b->jobs.size(), XFG_OK);
    std::lock_guard<std::mutex> g(c->qm);
    uint64_t t = c->next_ticket++;
    b->units_left = (int)units.size();
    c->pending[t] = std::move(bp);
    for (auto& u : units) {
        u.b = b;
        c->q.push_back(u);
    }
    c->qcv.notify_all();
    return t;
}

static std::unique_ptr<Batch> wait_batch(xfg_ctx* c, uint64_t t) {
    std::unique_lock<std::mutex> g(c->qm);
    auto it = c->pending.find(t);
    if (it == c->pending.end()) return nullptr;
    Batch* b = it->second.get();
    c->dcv.wait(g, [&] { return b->units_left == 0; });
    std::unique_ptr<Batch> bp = std::move(it->second);
    c->pending.erase(it);
    return bp;
}

static bool busy(xfg_ctx* c) {
    std::lock_guard<std::mutex> g(c->qm);
    return !c->pending.empty();
}

static int copy_out(xfg_ctx* c, const std::vector<uint8_t>& bytes, uint8_t* out, size_t* out_len) {
    if (!out_len) {
        c->err = "out_len is NULL";
        return XFG_INVALID_ARGUMENT;
    }
    if (!out || *out_len < bytes.size()) {
        *out_len = bytes.size();
        if (!out) return XFG_OK;
        c->err = "output buffer too small";
        return XFG_BUFFER_TOO_SMALL;
    }
    memcpy(out, bytes.data(), bytes.size());
    *out_len = bytes.size();
    return XFG_OK;
}

static int guarded(xfg_ctx* c, const std::function<int()>& f) {
    try {
        return f();
    } catch (const HipError& e) {
        c->err = e.what();
        return XFG_DEVICE_ERROR;
    } catch (const std::exception& e) {
        c->err = std::string("Prover error: ") + e.what();
        return XFG_PROVER_ERROR;
    }
}
}  // namespace xfg

using namespace xfg;

extern "C" {

xfg_ctx* xfg_ctx_create(int device_id) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device_id < 0 || device_id >= ndev) return nullptr;
    if (hipSetDevice(device_id) != hipSuccess) return nullptr;
    xfg_ctx* c = new xfg_ctx();
    c->device = device_id;
    try {
        lane0(c);
    } catch (...) {
        delete c;
        return nullptr;
    }
    return c;
}

void xfg_ctx_destroy(xfg_ctx* c) {
    if (!c) return;
    drain(c);
    {
        std::lock_guard<std::mutex> g(c->qm);
        c->stop = true;
        c->qcv.notify_all();
    }
    for (auto& t : c->workers) t.join();
    (void)hipSetDevice(c->device);
    for (auto& L : c->lanes) {
        (void)hipStreamSynchronize(L->stream);
        L->release();
        for (auto& e : L->ev) (void)hipEventDestroy(e);
        for (auto& e : L->lde_ev)
            if (e) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(L->stream);
        if (L->gstream) {
            (void)hipStreamSynchronize(L->gstream);
            (void)hipStreamDestroy(L->gstream);
        }
    }
    c->tables.tw.release();
    c->tables.pow7.release();
    c->tables.ipow7.release();
    for (auto& kv : c->tables.ce_div) kv.second.release();
    for (auto& kv : c->tables.four_buf) kv.second.release();
    for (auto& kv : c->tables.pass_buf) kv.second.release();
    delete c;
}

int xfg_default_options(xfg_options* o) {
    if (!o) return XFG_INVALID_ARGUMENT;
    // ProofOptions::new(42, 8, 4, FieldExtension::None, 8, 31) -- src/burn_mint_prover.rs:28-35
    *o = xfg_options{42, 8, 4, 1, 8, 31};
    return XFG_OK;
}

int xfg_last_error(const xfg_ctx* c, char* buf, size_t len) {
    if (!c) return XFG_INVALID_ARGUMENT;
    if (buf && len) {
        size_t k = std::min(len - 1, c->err.size());
        memcpy(buf, c->err.data(), k);
        buf[k] = 0;
    }
    return (int)c->err.size();
}

// Bytes of one serialised batch opening of `nu` leaves of an L-leaf tree (the u32 length, the u8
// vector count, one u8 length per vector, the digests): plan_batch_opening emits at most one node per
// distinct tree node at each level, so level j (2^j nodes) contributes at most min(nu, 2^j) digests.
static size_t opening_bound(u64 L, u64 nu) {
    size_t s = 4 + 1 + nu;
    for (unsigned j = 1; j <= ilog2(L); j++) s += 32 * std::min<u64>(nu, 1ULL << j);
    return s;
}

// The largest StarkProof::to_bytes this prover emits for (n, options), section by section as the
// serialiser below writes them, with nu = min(q, N) unique queries. Tight (configs[2]: 98.8 KB
// against ~78 KB proofs), so a fixed-size exchange record per proof costs little (bench.py).
size_t xfg_proof_size_bound(uint64_t n, const xfg_options* opts) {
    if (!opts || !is_pow2(n)) return 0;
    Opts o = to_opts(opts);
    if (o.fold < 2 || !is_pow2(o.fold) || o.beta == 0 || !is_pow2(o.beta)) return 0;
    const u64 N = n * o.beta, nu = std::min<u64>(o.q, N);
    const unsigned nl = num_fri_layers(N, o), lf = ilog2(o.fold);
    const size_t de = o.ext == 2 ? 2 : 1;
    const u64 rem_len = std::max<u64>(N >> (lf * nl) >> ilog2(o.beta), 1);
    size_t s = 7 + 9 + 6 + 1;                            // Context, num_unique_queries
    s += 2 + 32 * (size_t)(3 + nl);                      // commitments: trace, composition, layers, remainder
    s += 1 + 4 + nu * 7 * 8 + opening_bound(N, nu);      // trace queries
    s += 4 + nu * 8 * de + opening_bound(N, nu);         // constraint queries
    s += 2 + 1 + 14 * 8 * de + 2 + 8 * de;               // OOD frame
    s += 1;                                              // FRI layer count
    for (unsigned l = 0; l < nl; l++) s += 4 + nu * o.fold * 8 * de + opening_bound(N >> (lf * (l + 1)), nu);
    s += 2 + rem_len * 8 * de + 1 + 8;                   // remainder, partitions, pow nonce
    return s + 64;
}

int xfg_burn_air_consts(const xfg_burn_inputs* in, xfg_air_consts* out) {
    if (!in || !out) return XFG_INVALID_ARGUMENT;
    AirConst a;
    std::string err;
    int st = marshal(in, a, err);
    if (st) return st;
    memcpy(out->pub_inputs, a.pub, sizeof a.pub);
    out->nullifier = a.nullifier;
    out->commitment = a.commitment;
    return XFG_OK;
}

int xfg_prove_trace(xfg_ctx* c, const uint64_t* trace, uint32_t width, uint64_t n, const xfg_air_consts* air,
                    const xfg_options* opts, uint8_t* out, size_t* out_len) {
    if (!c) return XFG_INVALID_ARGUMENT;
    c->err.clear();
    if (!trace || !air || !opts || !out_len) {
        c->err = "null argument";
        return XFG_INVALID_ARGUMENT;
    }
    if (width != 7) {
        c->err = "XfgBurnMintAir traces have 7 columns";
        return XFG_INVALID_ARGUMENT;
    }
    Opts o = to_opts(opts);
    if (const char* m = check_options(n, o)) {
        c->err = std::string("Prover error: ") + m;
        return XFG_PROVER_ERROR;
    }
    for (u64 i = 0; i < 7 * n; i++)
        if (trace[i] >= P) {
            c->err = "trace element is not a canonical field element";
            return XFG_INVALID_ARGUMENT;
        }
    return guarded(c, [&]() -> int {
        HIPCHK(hipSetDevice(c->device));
        std::unique_ptr<Batch> bp(new Batch());
        bp->jobs.resize(1);
        ProofJob& j = bp->jobs[0];
        memset(&j.air, 0, sizeof(AirConst));
        memcpy(j.air.pub, air->pub_inputs, sizeof air->pub_inputs);
        j.air.nullifier = air->nullifier;
        j.air.commitment = air->commitment;
        bp->which = {0};
        bp->outs = {out};
        bp->out_lens = out_len;
        bp->trace_host = trace;
        bp->n = n;
        bp->o = o;
        bind_tables(c, bp.get());
        std::unique_ptr<Batch> b = wait_batch(c, enqueue(c, std::move(bp), {Unit{nullptr, 0, 1, -1}}));
        if (b->err) std::rethrow_exception(b->err);
        if (b->st[0] == XFG_PROVER_ERROR) {
            c->err = "Prover error: proof generation failed (degenerate transcript or DEEP degree)";
        } else if (b->st[0] == XFG_BUFFER_TOO_SMALL) {
            c->err = "output buffer too small";
        }
        return b->st[0];
    });
}

int xfg_prove_batch_submit(xfg_ctx* c, uint32_t count, const xfg_burn_inputs* inputs, uint64_t trace_length,
                           const xfg_options* opts, uint8_t* const* outs, size_t* out_lens, int* statuses,
                           uint64_t* ticket) {
    if (!c) return XFG_INVALID_ARGUMENT;
    c->err.clear();
    if (!inputs || !opts || !out_lens || !statuses || !ticket || count == 0) {
        c->err = count == 0 ? "empty batch" : "null argument";
        return XFG_INVALID_ARGUMENT;
    }
    *ticket = 0;
    u64 n = trace_length ? trace_length : 64;
    Opts o = to_opts(opts);
    if (const char* m = check_options(n, o)) {
        c->err = std::string("Prover error: ") + m;
        return XFG_PROVER_ERROR;
    }
    return guarded(c, [&]() -> int {
        HIPCHK(hipSetDevice(c->device));
        std::unique_ptr<Batch> bp(new Batch());
        // validation + marshalling (three Keccak-256 per proof) per input on the host pool: the
        // submitting thread is the start of every batch's latency
        std::vector<AirConst> airs(count);
        std::vector<std::string> errs(count);
        host_pool().parallel_for((int)count, [&](int i) { statuses[i] = marshal(&inputs[i], airs[i], errs[i]); });
        for (uint32_t i = 0; i < count; i++) {
            if (statuses[i]) {
                c->err = errs[i];
                continue;
            }
            bp->jobs.emplace_back();
            bp->jobs.back().air = airs[i];
            bp->which.push_back(i);
        }
        if (outs) bp->outs.assign(outs, outs + count);
        bp->out_lens = out_lens;
        bp->statuses = statuses;
        bp->n = n;
        bp->o = o;
        bind_tables(c, bp.get());
        std::vector<Unit> units = split_units(c, (int)bp->jobs.size());
        *ticket = enqueue(c, std::move(bp), std::move(units));
        return XFG_OK;
    });
}

int xfg_batch_wait(xfg_ctx* c, uint64_t ticket) {
    if (!c) return XFG_INVALID_ARGUMENT;
    return guarded(c, [&]() -> int {
        std::unique_ptr<Batch> b = wait_batch(c, ticket);
        if (!b) {
            c->err = "unknown batch ticket";
            return XFG_INVALID_ARGUMENT;
        }
        if (b->err) std::rethrow_exception(b->err);
        for (size_t k = 0; k < b->jobs.size(); k++) {
            b->statuses[b->which[k]] = b->st[k];
            if (b->st[k] == XFG_BUFFER_TOO_SMALL) c->err = "output buffer too small";
            if (b->st[k] == XFG_PROVER_ERROR)
                c->err = "Prover error: proof generation failed (degenerate transcript or DEEP degree)";
        }
        return XFG_OK;
    });
}

int xfg_prove_batch(xfg_ctx* c, uint32_t count, const xfg_burn_inputs* inputs, uint64_t trace_length,
                    const xfg_options* opts, uint8_t* const* outs, size_t* out_lens, int* statuses) {
    uint64_t t = 0;
    int r = xfg_prove_batch_submit(c, count, inputs, trace_length, opts, outs, out_lens, statuses, &t);
    if (r) return r;
    return xfg_batch_wait(c, t);
}

int xfg_prepare(xfg_ctx* c, uint32_t count, uint64_t trace_length, const xfg_options* opts) {
    if (!c || !opts || count == 0) return XFG_INVALID_ARGUMENT;
    c->err.clear();
    u64 n = trace_length ? trace_length : 64;
    Opts o = to_opts(opts);
    if (const char* m = check_options(n, o)) {
        c->err = std::string("Prover error: ") + m;
        return XFG_PROVER_ERROR;
    }
    return guarded(c, [&]() -> int {
        HIPCHK(hipSetDevice(c->device));
        // two throw-away proving passes over a fixed valid statement size every lane workspace
        // (device + pinned host) and load every code object; nothing is cached between proofs
        xfg_burn_inputs in{};
        in.burn_amount = in.mint_amount = STANDARD_BURN;
        for (int i = 0; i < 32; i++) in.tx_prefix_hash[i] = (uint8_t)(i + 1);
        static const uint8_t rcpt[20] = {1}, sec[32] = {2};
        in.recipient_address = rcpt;
        in.recipient_len = 20;
        in.secret = sec;
        in.secret_len = 32;
        in.network_id = 1;
        in.target_chain_id = 42161;
        in.commitment_version = 1;
        AirConst a;
        std::string err;
        if (marshal(&in, a, err)) return XFG_PROVER_ERROR;
        // every lane proves one full unit, twice (lane-pinned units)
        ensure_workers(c);
        const int nl = (int)c->workers.size(), U = std::min<int>((int)count, unit_size());
        for (int pass = 0; pass < 2; pass++) {
            std::unique_ptr<Batch> bp(new Batch());
            bp->jobs.resize((size_t)nl * U);
            for (auto& j : bp->jobs) j.air = a;
            bp->n = n;
            bp->o = o;
            bind_tables(c, bp.get());
            std::vector<Unit> units;
            for (int l = 0; l < nl; l++) units.push_back(Unit{nullptr, l * U, (l + 1) * U, l});
            std::unique_ptr<Batch> b = wait_batch(c, enqueue(c, std::move(bp), std::move(units)));
            if (b->err) std::rethrow_exception(b->err);
        }
        HIPCHK(hipDeviceSynchronize());
        return XFG_OK;
    });
}

int xfg_prove_burn_mint(xfg_ctx* c, const xfg_burn_inputs* in, uint64_t trace_length, const xfg_options* opts,
                        uint8_t* out, size_t* out_len) {
    if (!c) return XFG_INVALID_ARGUMENT;
    if (!out_len) return XFG_INVALID_ARGUMENT;
    int st = 0;
    uint8_t* outs[1] = {out};
    size_t lens[1] = {*out_len};
    int r = xfg_prove_batch(c, 1, in, trace_length, opts, outs, lens, &st);
    if (r) return r;
    *out_len = lens[0];
    return st;
}

int xfg_selftest_field(uint64_t a, uint64_t b, uint64_t* out3) {
    if (!out3 || a >= P || b >= P) return XFG_INVALID_ARGUMENT;
    out3[0] = gl_mul(a, b);
    out3[1] = gl_add(a, b);
    out3[2] = gl_sub(a, b);
    return XFG_OK;
}

int xfg_set_timing(xfg_ctx* c, int enabled) {
    if (!c) return XFG_INVALID_ARGUMENT;
    c->timing = enabled != 0;
    for (auto& L : c->lanes) L->timing = c->timing;
    return XFG_OK;
}

int xfg_stage_times(const xfg_ctx* c, double* ms, const char** names, int max) {
    if (!c) return 0;
    int k = std::min<int>(max, ST_COUNT);
    for (int i = 0; i < k; i++) {
        if (ms) ms[i] = c->lanes.empty() ? 0.0 : c->lanes[c->last_lane]->stage_ms[i];
        if (names) names[i] = STAGE_NAMES[i];
    }
    return k;
}

int xfg_bench_lde(xfg_ctx* c, uint32_t count, uint64_t n, uint32_t blowup, uint32_t iters, double* avg_ms) {
    if (!c || !avg_ms || !is_pow2(n) || !is_pow2(blowup) || n < 8 || blowup < 2 || blowup > 16 || iters == 0)
        return XFG_INVALID_ARGUMENT;
    if (busy(c)) {  // lane 0's stream and buffers belong to the workers while batches are pending
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        const int logn = (int)ilog2(n), logbeta = (int)ilog2(blowup);
        const u64 N = n * blowup;
        ensure_tables(c, logn + logbeta);
        ensure_fourstep(c, logn, logbeta);
        Tables T = tables_of(c);
        L->coef.ensure((size_t)count * 7 * n);
        L->scratch.ensure((size_t)count * 7 * N);
        L->lde.ensure((size_t)count * 7 * N);
        // deterministic canonical coefficients
        std::vector<u64> h((size_t)count * 7 * n);
        u64 x = 0x46472d535441524bULL;  // "FG-STARK"
        for (auto& v : h) {
            x += 0x9E3779B97F4A7C15ULL;
            u64 z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
            v = (z ^ (z >> 31)) % P;
        }
        HIPCHK(hipMemcpy(L->coef.p, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        launch_lde(L->coef.p, n, L->lde.p, L->scratch.p, count * 7, logn, logbeta, T, L->stream);  // warm
        HIPCHK(hipEventRecord(L->ev[0], L->stream));
        for (uint32_t i = 0; i < iters; i++)
            launch_lde(L->coef.p, n, L->lde.p, L->scratch.p, count * 7, logn, logbeta, T, L->stream);
        HIPCHK(hipEventRecord(L->ev[1], L->stream));
        HIPCHK(hipEventSynchronize(L->ev[1]));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, L->ev[0], L->ev[1]));
        *avg_ms = ms / iters;
        return XFG_OK;
    });
}

int xfg_lde_probe(xfg_ctx* c, int enabled, double* total_ms, uint64_t* launch_sets, uint64_t* polys) {
    if (!c) return XFG_INVALID_ARGUMENT;
    if (busy(c)) {  // lane counters belong to the workers while batches are pending
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    double ms = 0;
    u64 sets = 0, np = 0;
    for (auto& L : c->lanes) {
        ms += L->lde_ms;
        sets += L->lde_sets;
        np += L->lde_polys;
        if (enabled) L->lde_ms = 0, L->lde_sets = 0, L->lde_polys = 0;
        L->lde_probe = enabled != 0;
    }
    if (total_ms) *total_ms = ms;
    c->lde_probe = enabled != 0;
    if (launch_sets) *launch_sets = sets;
    if (polys) *polys = np;
    return XFG_OK;
}

int xfg_debug_lde(xfg_ctx* c, const uint64_t* coef, uint32_t npoly, uint64_t n, uint32_t blowup, uint64_t* out) {
    if (!c || !coef || !out || !is_pow2(n) || !is_pow2(blowup) || n < 8 || blowup < 2 || blowup > 16)
        return XFG_INVALID_ARGUMENT;
    if (busy(c)) {  // lane 0's stream and buffers belong to the workers while batches are pending
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        const int logn = (int)ilog2(n), logbeta = (int)ilog2(blowup);
        const u64 N = n * blowup;
        ensure_tables(c, logn + logbeta);
        ensure_fourstep(c, logn, logbeta);
        Tables T = tables_of(c);
        L->coef.ensure((size_t)npoly * n);
        L->scratch.ensure((size_t)npoly * N);
        L->lde.ensure((size_t)npoly * N);
        HIPCHK(hipMemcpy(L->coef.p, coef, (size_t)npoly * n * 8, hipMemcpyHostToDevice));
        launch_lde(L->coef.p, n, L->lde.p, L->scratch.p, npoly, logn, logbeta, T, L->stream);
        std::vector<u64> cm((size_t)npoly * N);
        HIPCHK(hipMemcpyAsync(cm.data(), L->lde.p, cm.size() * 8, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipStreamSynchronize(L->stream));
        for (u64 p = 0; p < npoly; p++)  // coset-major -> natural order
            for (u64 t = 0; t < blowup; t++)
                for (u64 m = 0; m < n; m++) out[p * N + t + blowup * m] = cm[(p * blowup + t) * n + m];
        return XFG_OK;
    });
}

int xfg_debug_interpolate(xfg_ctx* c, const uint64_t* evals, uint32_t npoly, uint64_t n, int offset7, uint64_t* out) {
    if (!c || !evals || !out || !is_pow2(n) || n < 8) return XFG_INVALID_ARGUMENT;
    if (busy(c)) {  // lane 0's stream and buffers belong to the workers while batches are pending
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        const int logn = (int)ilog2(n);
        ensure_tables(c, std::max(logn, c->tables.LM));
        if (logn >= 4) ensure_fourstep(c, logn - 1, 1);  // inverse tables up to size n
        Tables T = tables_of(c);
        L->trace.ensure((size_t)npoly * n);
        L->coef.ensure((size_t)npoly * n);
        L->scratch.ensure((size_t)npoly * n);
        HIPCHK(hipMemcpy(L->trace.p, evals, (size_t)npoly * n * 8, hipMemcpyHostToDevice));
        launch_interpolate(L->trace.p, n, L->coef.p, n, L->scratch.p, npoly, logn, offset7 != 0, n, T, L->stream);
        HIPCHK(hipMemcpyAsync(out, L->coef.p, (size_t)npoly * n * 8, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipStreamSynchronize(L->stream));
        return XFG_OK;
    });
}

int xfg_debug_field(xfg_ctx* c, uint32_t op, uint64_t count, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    if (!c || !a || !b || !out || op > 8 || count == 0) return XFG_INVALID_ARGUMENT;
    if (busy(c)) {
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        L->trace.ensure((size_t)count * 3);
        u64* da = L->trace.p;
        u64* db = da + count;
        u64* dout = db + count;
        HIPCHK(hipMemcpy(da, a, count * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(db, b, count * 8, hipMemcpyHostToDevice));
        launch_field_op((int)op, da, db, dout, count, L->stream);
        HIPCHK(hipMemcpyAsync(out, dout, count * 8, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipStreamSynchronize(L->stream));
        return XFG_OK;
    });
}

int xfg_debug_coin_draws(xfg_ctx* c, const uint32_t seed[8], uint64_t counter, uint32_t k, uint32_t ext,
                         const uint64_t reject[4], uint64_t* out_wave, uint64_t* out_seq, uint64_t counters[2],
                         int ok[2]) {
    if (!c || !seed || !reject || !out_wave || !out_seq || !counters || !ok || k == 0 || k > 64 ||
        (ext != 1 && ext != 2))
        return XFG_INVALID_ARGUMENT;
    if (busy(c)) {
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        L->trace.ensure(4 + 4 * (size_t)k + 2 + 1);
        u64* drej = L->trace.p;
        u64* dw = drej + 4;
        u64* ds = dw + 2 * k;
        u64* dctr = ds + 2 * k;
        int* dok = (int*)(dctr + 2);
        HIPCHK(hipMemcpy(drej, reject, 32, hipMemcpyHostToDevice));
        HIPCHK(hipMemset(dw, 0, 16 * (size_t)k));
        DevCoin c0;
        memcpy(c0.seed.w, seed, 32);
        c0.counter = counter;
        c0.pad = 0;
        launch_coin_draw_test(c0, (int)k, (int)ext, drej, dw, ds, dctr, dok, L->stream);
        HIPCHK(hipMemcpyAsync(out_wave, dw, 16 * (size_t)k, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipMemcpyAsync(out_seq, ds, 16 * (size_t)k, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipMemcpyAsync(counters, dctr, 16, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipMemcpyAsync(ok, dok, 8, hipMemcpyDeviceToHost, L->stream));
        HIPCHK(hipStreamSynchronize(L->stream));
        return XFG_OK;
    });
}

int xfg_debug_ood_deep(xfg_ctx* c, uint32_t count, uint64_t n, const uint64_t* coef, const uint64_t* hcoef,
                       const uint64_t* zpts, const uint64_t* coeffs, uint64_t* ood_out, uint64_t* deep_out) {
    if (!c || !coef || !hcoef || !zpts || !coeffs || !ood_out || !deep_out || !is_pow2(n) || n < 8 || count == 0)
        return XFG_INVALID_ARGUMENT;
    if (busy(c)) {
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        Lane* L = lane0(c);
        HIPCHK(hipSetDevice(c->device));
        const int logn = (int)ilog2(n);
        const size_t B = count;
        L->coef.ensure(B * 7 * n);
        L->hcoef.ensure(B * n);
        L->zpts.ensure(B * 2);
        L->partial.ensure(B * 15 * ood_partial_count(logn));
        L->carry.ensure(B * 2 * ood_partial_count(logn));
        L->ood.ensure(B * 15);
        L->deep.ensure(B * n);
        L->dp.ensure(B);
        hipStream_t s = L->stream;
        HIPCHK(hipMemcpyAsync(L->coef.p, coef, B * 7 * n * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(L->hcoef.p, hcoef, B * n * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(L->zpts.p, zpts, B * 2 * 8, hipMemcpyHostToDevice, s));
        launch_ood(L->coef.p, L->hcoef.p, L->zpts.p, L->partial.p, L->ood.p, logn, (int)B, 1, s);
        HIPCHK(hipMemcpyAsync(ood_out, L->ood.p, B * 15 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<DeepParams> dps(B);
        for (size_t b = 0; b < B; b++) {  // as prove_lane: c1, c2 from the OOD values
            DeepParams& P = dps[b];
            memset(&P, 0, sizeof P);
            for (int k = 0; k < 7; k++) P.a[k][0] = coeffs[b * 8 + k];
            P.gamma[0] = coeffs[b * 8 + 7];
            P.z[0] = zpts[2 * b];
            P.zg[0] = zpts[2 * b + 1];
            P.zinv[0] = gl_inv(P.z[0]);
            P.zginv[0] = gl_inv(P.zg[0]);
            const u64* o = ood_out + b * 15;
            u64 c1 = gl_mul(P.gamma[0], o[14]), c2 = 0;
            for (int k = 0; k < 7; k++) {
                c1 = gl_add(c1, gl_mul(P.a[k][0], o[2 * k]));
                c2 = gl_add(c2, gl_mul(P.a[k][0], o[2 * k + 1]));
            }
            P.c1[0] = c1;
            P.c2[0] = c2;
        }
        HIPCHK(hipMemcpyAsync(L->dp.p, dps.data(), B * sizeof(DeepParams), hipMemcpyHostToDevice, s));
        launch_deep(L->coef.p, L->hcoef.p, L->dp.p, L->partial.p, L->carry.p, L->deep.p, logn, (int)B, 1, s);
        HIPCHK(hipMemcpyAsync(deep_out, L->deep.p, B * n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return XFG_OK;
    });
}

int xfg_verify_batch_gpu(xfg_ctx* c, uint32_t count, const uint8_t* const* proofs, const size_t* lens,
                         const xfg_air_consts* airs, const xfg_options* acceptable, int* results) {
    if (!c || !proofs || !lens || !airs || !acceptable || !results) return XFG_INVALID_ARGUMENT;
    c->err.clear();
    if (busy(c)) {
        c->err = "batches pending: call xfg_batch_wait first";
        return XFG_INVALID_ARGUMENT;
    }
    return guarded(c, [&]() -> int {
        HIPCHK(hipSetDevice(c->device));
        const Opts acc = to_opts(acceptable);
        HostTrace ht;
        ht.mark("start");
        // per-proof transcript states and plan fragments are kept in the context between calls
        // (reset in place: a large batch would otherwise allocate and free ~10^5 small blocks)
        auto& V = c->vb;
        if (V.st.size() < count) V.st.resize(count);
        if (V.frag.size() < count) V.frag.resize(count);
        std::vector<VState>& st = V.st;
        std::vector<std::string> err(count);
        // per-proof host phases on the host pool (spawning 16 threads per phase cost more than the
        // phases' own work at 64 proofs); a proof per task
        auto parallel = [&](const std::function<void(uint32_t)>& f) {
            host_pool().parallel_for((int)count, [&](int i) { f((uint32_t)i); });
        };
        // 1. transcripts (host threads)
        parallel([&](uint32_t i) {
            if (!proofs[i]) {
                err[i] = "null proof";
                return;
            }
            try {
                err[i] = verify_transcript(proofs[i], lens[i], air_of(&airs[i]), acc, st[i]);
            } catch (const std::exception& e) {
                err[i] = std::string("ProofDeserializationError(\"") + e.what() + "\")";
            }
        });
        ht.mark("transcripts");
        // 2. plan: per-proof fragments (openings, queries) built in parallel; blob offsets by prefix
        //    sum of the accepted proofs' lengths
        std::vector<size_t> boff(count + 1, 0);
        for (uint32_t i = 0; i < count; i++) boff[i + 1] = boff[i] + (err[i].empty() ? lens[i] : 0);
        std::vector<VerifyPlan>& frag = V.frag;
        parallel([&](uint32_t i) {
            if (!err[i].empty()) return;
            std::string e;
            if (!plan_proof(st[i], boff[i], frag[i], e)) err[i] = e;
        });
        ht.mark("plan_fragments");
        // 3. concatenate into one pinned staging region (parallel fill) and one DMA
        struct Off {
            size_t t = 0, lf = 0, v = 0, q = 0, fp = 0;
        };
        std::vector<Off> fo(count + 1);
        std::vector<int> planned(count, -1);
        for (uint32_t i = 0; i < count; i++) {
            const bool ok = err[i].empty();
            const VerifyPlan& f = frag[i];
            Off& a = fo[i];
            Off& b = fo[i + 1];
            b.t = a.t + (ok ? f.trees.size() : 0);
            b.lf = a.lf + (ok ? f.tleaves.size() : 0);
            b.v = a.v + (ok ? f.vecs.size() : 0);
            b.q = a.q + (ok ? f.fqueries.size() : 0);
            b.fp = a.fp + (ok ? 1 : 0);
            if (ok) planned[i] = (int)a.fp;
        }
        const Off& E = fo[count];
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_blob = 0, o_t = al(boff[count]), o_lf = al(o_t + E.t * sizeof(VTree)),
                     o_v = al(o_lf + E.lf * sizeof(VTreeLeaf)), o_fp = al(o_v + E.v * sizeof(VVec)),
                     o_fq = al(o_fp + E.fp * sizeof(VFieldProof)), total_b = al(o_fq + E.q * sizeof(VFieldQuery));
        uint8_t* H = V.stage.ensure(total_b);
        VTree* ht_ = (VTree*)(H + o_t);
        VTreeLeaf* hlf = (VTreeLeaf*)(H + o_lf);
        VVec* hv = (VVec*)(H + o_v);
        VFieldProof* hfp = (VFieldProof*)(H + o_fp);
        VFieldQuery* hfq = (VFieldQuery*)(H + o_fq);
        parallel([&](uint32_t i) {
            if (planned[i] < 0) return;
            memcpy(H + o_blob + boff[i], proofs[i], lens[i]);
            const VerifyPlan& f = frag[i];
            const Off& a = fo[i];
            for (size_t k = 0; k < f.trees.size(); k++) {
                VTree t = f.trees[k];
                t.leaf0 += (uint32_t)a.lf;
                t.vec0 += (uint32_t)a.v;
                t.proof = (uint32_t)a.fp;
                ht_[a.t + k] = t;
            }
            memcpy(hlf + a.lf, f.tleaves.data(), f.tleaves.size() * sizeof(VTreeLeaf));
            memcpy(hv + a.v, f.vecs.data(), f.vecs.size() * sizeof(VVec));
            hfp[a.fp] = f.fproof;
            for (size_t k = 0; k < f.fqueries.size(); k++) {
                hfq[a.q + k] = f.fqueries[k];
                hfq[a.q + k].proof = (uint32_t)a.fp;
            }
        });
        ht.mark("plan_merge");
        std::vector<uint32_t> flags(E.fp, 0);
        if (E.fp > 0) {
            hipStream_t s = lane0(c)->stream;
            V.dstage.ensure(total_b);
            V.flags.ensure(E.fp);
            HIPCHK(hipMemcpyAsync(V.dstage.p, H, total_b, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemsetAsync(V.flags.p, 0, E.fp * 4, s));
            ht.mark("upload_enqueue");
            uint8_t* D = V.dstage.p;
            launch_verify(D + o_blob, (const VTree*)(D + o_t), E.t, (const VTreeLeaf*)(D + o_lf), (const VVec*)(D + o_v),
                          (const VFieldProof*)(D + o_fp), (const VFieldQuery*)(D + o_fq), E.q, V.flags.p, s);
            HIPCHK(hipMemcpyAsync(flags.data(), V.flags.p, flags.size() * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            ht.mark("device");
        }
        // 4. verdicts in the host verifier's check order
        parallel([&](uint32_t i) {
            if (planned[i] >= 0) err[i] = finish_proof(st[i], flags[planned[i]]);
            results[i] = proofs[i] ? (err[i].empty() ? XFG_OK : XFG_VERIFY_FAILED) : XFG_INVALID_ARGUMENT;
        });
        ht.mark("finish");
        ht.dump((int)count);
        return XFG_OK;
    });
}

}  // extern "C"
