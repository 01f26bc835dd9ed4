// Proof parsing (StarkProof::from_bytes) and the STARK verifier for the burn AIR, host C++.
//
// Replaces winterfell::verify::<XfgBurnMintAir, Blake3_256, DefaultRandomCoin> as called by the
// reference verifier (src/burn_mint_verifier.rs:265-283; batch loops :326-338, :386-408). The
// statement is the 12 public inputs plus the two Keccak-derived AIR constants (nullifier,
// commitment): the corrected AIR binds the prover's secret through them,
// so the verifier takes them as inputs instead of rebuilding the AIR from a fixed secret.
// Product code: independent of the oracle under oracle/ (which is test infrastructure only).
#include <hip/hip_runtime.h>

#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "verifier.hpp"

namespace xfg {

// ------------------------------------------------------------------ byte reader
struct Reader {
    const uint8_t* p;
    size_t n, off = 0;
    bool bad = false;
    const uint8_t* take(size_t k) {
        if (bad || k > n - off) {
            bad = true;
            return nullptr;
        }
        const uint8_t* q = p + off;
        off += k;
        return q;
    }
    u64 u(int bytes) {
        const uint8_t* q = take((size_t)bytes);
        u64 v = 0;
        if (q)
            for (int i = 0; i < bytes; i++) v |= (u64)q[i] << (8 * i);
        return v;
    }
};
// BatchMerkleProof node vectors inside a paths byte vector (u8 vector count, per vector u8 count +
// digests): the content parse of VerifierChannel::new, after the options check
static bool parse_paths(const Span& raw, Paths& out) {
    Reader s{raw.p, raw.n};
    const u64 m = s.u(1);
    out.ptr.resize(m);
    out.cnt.resize(m);
    for (u64 i = 0; i < m; i++) {
        const u64 c = s.u(1);
        const uint8_t* d = s.take(c * 32);
        if (!d) return false;
        out.ptr[i] = d;
        out.cnt[i] = (uint32_t)c;
    }
    return !s.bad && s.off == raw.n;
}
static bool read_span(Reader& r, int len_bytes, Span& s) {
    s.n = r.u(len_bytes);
    s.p = r.take(s.n);
    return !r.bad;
}
// every field element of a proof must be canonical: winter-math 0.8 BaseElement::read_from rejects
// a value >= p. Winterfell reads the element sections (queries, OOD frame, FRI layers, remainder)
// only in VerifierChannel::new, after the acceptable-options check, so parse_proof (from_bytes)
// stays structural and verify_transcript runs this check after the options (the field code of
// the host and GPU verifiers then assumes canonical operands)
static bool canonical_elems(const Span& s) {
    if (s.n % 8) return false;
    for (size_t i = 0; i < s.n / 8; i++)
        if (s.elem(i) >= P) return false;
    return true;
}

// returns "" on success, else the ProofDeserializationError text
std::string parse_proof(const uint8_t* bytes, size_t len, ParsedProof& pf) {
    Reader r{bytes, len};
    pf.base = bytes;
    pf.width = r.u(1);
    pf.aux = r.u(1);
    pf.logn = r.u(1);
    const u64 meta = r.u(2);
    r.take(meta);
    const u64 mlen = r.u(1), modulus = r.u(8);
    pf.o.q = r.u(1);
    pf.o.beta = r.u(1);
    pf.o.grind = r.u(1);
    pf.o.ext = r.u(1);
    pf.o.fold = r.u(1);
    pf.o.remdeg = r.u(1);
    if (r.bad) return "ProofDeserializationError(\"context: unexpected end of input\")";
    if (mlen != 8 || modulus != xfg::P) return "InconsistentBaseField";
    if (pf.logn < 3 || pf.logn > 32) return "ProofDeserializationError(\"context: invalid trace length\")";
    // FieldExtension::{None, Quadratic, Cubic} = 1, 2, 3 (winter-air 0.8 ProofOptions::read_from)
    if (pf.o.ext < 1 || pf.o.ext > 3) return "ProofDeserializationError(\"context: invalid field extension\")";
    pf.num_unique = r.u(1);
    const u64 clen = r.u(2);
    const uint8_t* c = r.take(clen);
    if (!c || clen % 32) return "ProofDeserializationError(\"commitments\")";
    pf.com.resize(clen / 32);
    pf.com_p = c;
    if (clen) memcpy(pf.com.data(), c, clen);  // (an empty vector's data() may be null)
    if (r.u(1) != 1) return "ProofDeserializationError(\"trace queries: expected one segment\")";
    // StarkProof::read_from keeps every section below as a byte vector; their contents (Merkle node
    // vectors, the OOD frame layout, the remainder's element size) are parsed by parse_contents
    // after the acceptable-options check, as VerifierChannel::new does
    if (!read_span(r, 4, pf.trace_rows) || !read_span(r, 4, pf.trace_paths_raw))
        return "ProofDeserializationError(\"trace queries\")";
    if (!read_span(r, 4, pf.constraint_rows) || !read_span(r, 4, pf.constraint_paths_raw))
        return "ProofDeserializationError(\"constraint queries\")";
    if (!read_span(r, 2, pf.ood_raw) || !read_span(r, 2, pf.hz)) return "ProofDeserializationError(\"OOD frame\")";
    const u64 nl = r.u(1);
    pf.fri_vals.resize(nl);
    pf.fri_paths_raw.resize(nl);
    for (u64 l = 0; l < nl; l++)
        if (!read_span(r, 4, pf.fri_vals[l]) || !read_span(r, 4, pf.fri_paths_raw[l]))
            return "ProofDeserializationError(\"FRI layer\")";
    if (!read_span(r, 2, pf.fri_rem)) return "ProofDeserializationError(\"FRI remainder\")";
    pf.partitions = r.u(1);
    pf.nonce = r.u(8);
    if (r.bad) return "ProofDeserializationError(\"unexpected end of input\")";
    if (r.off != len) return "ProofDeserializationError(\"trailing bytes\")";
    pf.size = r.off;
    return "";
}

// VerifierChannel::new's content parse of the byte-vector sections: "" or the
// ProofDeserializationError
std::string parse_contents(ParsedProof& pf) {
    const size_t esz = 8 * (size_t)pf.o.ext;  // bytes per E element
    if (!parse_paths(pf.trace_paths_raw, pf.trace_paths)) return "ProofDeserializationError(\"trace query paths\")";
    if (!parse_paths(pf.constraint_paths_raw, pf.constraint_paths))
        return "ProofDeserializationError(\"constraint query paths\")";
    // frame of two rows (current, next) of `width` E values each: exactly that many, so every
    // reader of the frame stays inside the proof bytes
    if (pf.ood_raw.n != 1 + 2 * pf.width * esz || pf.ood_raw.p[0] != 2 || pf.hz.n != esz)
        return "ProofDeserializationError(\"OOD frame layout\")";
    pf.ood = Span{pf.ood_raw.p + 1, pf.ood_raw.n - 1};
    pf.fri_paths.resize(pf.fri_paths_raw.size());
    for (size_t l = 0; l < pf.fri_paths_raw.size(); l++)
        if (!parse_paths(pf.fri_paths_raw[l], pf.fri_paths[l])) return "ProofDeserializationError(\"FRI layer paths\")";
    if (pf.fri_rem.n % esz) return "ProofDeserializationError(\"FRI remainder\")";
    return "";
}

// ------------------------------------------------------------------ batch Merkle root
// BatchMerkleProof::get_root: node vector i must hold at least the siblings the opening plan of
// `idx` takes from it, in that order; every node on the way to the root is then recomputed, level by
// level. Nodes past the ones the walk takes are ignored: winter-crypto 0.8's get_root consumes the
// vectors through per-position pointers and never checks that every node was used (the oracle's
// batch_root restates the same walk, oracle/orc_stark.c), so an opening with a trailing extra node
// still verifies there, and here. PARITY UNPINNED against upstream: winter-crypto 0.8.x
// (`BatchMerkleProof::get_root`, src/merkle/proofs.rs of that crate) is not vendored in the reference
// and no reference fixture covers an over-long node vector, so this acceptance rests on the
// restatement of its published walk (the per-position `proof_pointers` advance, no final check that
// each vector was consumed); test_gpu_batch_verify_node_vector_mutants pins GPU = host = oracle only.
bool merkle_symbolic(const std::vector<u64>& idx, const Paths& paths, u64 L, MerkleSym& out) {
    thread_local BatchOpening plan;
    plan_batch_opening(idx, L, plan);
    // reset in place: callers reuse `out`, so steady-state planning does not allocate
    out.nslots = out.root = 0;
    out.leaf_slot.clear();
    out.given.clear();
    for (auto& v : out.levels) v.clear();
    if (plan.size() != paths.ptr.size()) return false;
    const unsigned depth = ilog2(L);
    // nodes available per level (0 = leaves) as (heap index, slot), sorted before use; per-thread
    // scratch so batch planning does not allocate per tree
    thread_local std::vector<std::vector<std::pair<u64, uint32_t>>> lv;
    if (lv.size() < depth + 1) lv.resize(depth + 1);
    for (unsigned l = 0; l <= depth; l++) lv[l].clear();
    uint32_t s = 0;
    out.leaf_slot.resize(idx.size());
    for (size_t i = 0; i < idx.size(); i++) {
        out.leaf_slot[i] = s;
        lv[0].push_back({L + idx[i], s++});
    }
    for (size_t i = 0; i < plan.size(); i++) {
        if (paths.cnt[i] < plan.len[i]) return false;
        for (unsigned k = 0; k < plan.len[i]; k++) {
            const u64 h = plan.row(i)[k];
            lv[depth - (63 - __builtin_clzll(h))].push_back({h, s});
            out.given.push_back({s++, paths.ptr[i] + 32 * k});
        }
    }
    thread_local std::vector<u64> level, up;
    level.resize(idx.size());
    for (size_t i = 0; i < idx.size(); i++) level[i] = L + idx[i];
    std::sort(level.begin(), level.end());
    level.erase(std::unique(level.begin(), level.end()), level.end());
    if (out.levels.size() < depth) out.levels.resize(depth);
    out.nlev = depth;
    for (unsigned l = 0; l < depth; l++) {
        auto& cur = lv[l];
        std::sort(cur.begin(), cur.end());
        for (size_t i = 1; i < cur.size(); i++)
            if (cur[i].first == cur[i - 1].first) return false;
        auto find = [&](u64 h, uint32_t& sl) {
            auto it = std::lower_bound(cur.begin(), cur.end(), std::make_pair(h, (uint32_t)0));
            if (it == cur.end() || it->first != h) return false;
            sl = it->second;
            return true;
        };
        std::vector<uint32_t>& trip = out.levels[l];
        trip.reserve(3 * level.size());
        up.clear();
        for (u64 x : level) {
            const u64 p = x >> 1;
            if (!up.empty() && up.back() == p) continue;
            uint32_t a, b;
            if (!find(2 * p, a) || !find(2 * p + 1, b)) return false;
            trip.insert(trip.end(), {s, a, b});
            lv[l + 1].push_back({p, s++});
            up.push_back(p);
        }
        level.swap(up);
    }
    if (level.size() != 1 || level[0] != 1) return false;
    out.root = lv[depth].back().second;  // the last node added at the top level is the root
    for (auto& e : lv[depth])
        if (e.first == 1) out.root = e.second;
    out.nslots = s;
    return true;
}
static bool batch_root(const std::vector<u64>& idx, const std::vector<Digest>& leaf, const Paths& paths, u64 L,
                       Digest& root) {
    MerkleSym sym;
    if (!merkle_symbolic(idx, paths, L, sym)) return false;
    std::vector<Digest> val(sym.nslots);
    for (size_t i = 0; i < idx.size(); i++) val[sym.leaf_slot[i]] = leaf[i];
    for (auto& g : sym.given) memcpy(val[g.first].w, g.second, 32);
    for (unsigned l = 0; l < sym.nlev; l++) {
        const auto& lvl = sym.levels[l];
        for (size_t t = 0; t < lvl.size(); t += 3) val[lvl[t]] = b3_merge(val[lvl[t + 1]], val[lvl[t + 2]]);
    }
    root = val[sym.root];
    return true;
}
static bool same(const Digest& a, const Digest& b) { return !memcmp(a.w, b.w, 32); }
static Digest leaf_hash(const uint8_t* bytes, size_t len) { return blake3_bytes(bytes, len); }

// ------------------------------------------------------------------ burn AIR at a point
// evaluate_transition (src/burn_mint_air.rs:335-378, corrected AIR A.2) and the 8 assertions
// (:380-395, final state assertion at n - 1)
// evaluated over E (the OOD frame is E-valued with a field extension; base values have b = 0)
static void air_transition(const AirConst& a, const E2 cur[7], const E2 nxt[7], E2 r[7]) {
    const u64 std_burn = 8000000ULL, large = gl_mul(std_burn, 1000);
    r[0] = e2_mul(e2_sub(cur[0], e2(std_burn)), e2_sub(cur[0], e2(large)));
    r[1] = e2_sub(cur[1], cur[0]);
    r[2] = e2_sub(cur[2], e2(a.pub[2]));
    r[3] = e2_sub(cur[3], e2(a.pub[3]));
    const E2 d = e2_sub(nxt[4], cur[4]);
    r[4] = e2_mul(d, e2_sub(d, e2(1)));
    r[5] = e2_sub(cur[5], e2(a.nullifier));
    r[6] = e2_sub(cur[6], e2(a.commitment));
}

// FRI apply_drp on one row (folding 8, domain offset 7): interpolate the 8 values on the coset
// x * <w_8> (per coordinate: base-field weights) and evaluate at alpha
static E2 fold_row(const E2 v[8], u64 x, E2 alpha) {
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
// E element i of a span of DE-coordinate elements
static E2 elem_e(const Span& s, size_t i, int de) { return de == 2 ? E2{s.elem(2 * i), s.elem(2 * i + 1)} : e2(s.elem(i)); }

// returns "" when the proof verifies, else the VerifierError (Debug form)
std::string verify_transcript(const uint8_t* bytes, size_t len, const AirConst& air, const Opts& acceptable,
                              VState& st) {
    ParsedProof& pf = st.pf;
    std::string e = parse_proof(bytes, len, pf);
    if (!e.empty()) return e;
    if (pf.width != 7 || pf.aux != 0) return "InconsistentTraceWidth";
    const Opts& o = pf.o;
    if (memcmp(&o, &acceptable, sizeof o)) return "UnacceptableProofOptions";  // AcceptableOptions::OptionSet
    const u64 n = 1ULL << pf.logn;
    if (check_options(n, o)) return "UnacceptableProofOptions";
    // VerifierChannel::new: the section contents and the element sections are deserialised now
    e = parse_contents(pf);
    if (!e.empty()) return e;
    bool canon = canonical_elems(pf.trace_rows) && canonical_elems(pf.constraint_rows) && canonical_elems(pf.ood) &&
                 canonical_elems(pf.hz) && canonical_elems(pf.fri_rem);
    for (const Span& v : pf.fri_vals) canon = canon && canonical_elems(v);
    if (!canon) return "ProofDeserializationError(\"invalid field element\")";
    const int de = (int)o.ext;  // E = base field (1) or its quadratic extension (2)
    const u64 beta = o.beta, N = n * beta;
    const unsigned nl = num_fri_layers(N, o);
    if (pf.com.size() != 3 + nl || pf.fri_vals.size() != nl || pf.partitions != 0 || pf.num_unique == 0 ||
        pf.ood.n != 14 * 8 * (size_t)de)
        return "ProofDeserializationError(\"inconsistent proof structure\")";
    const u64 nu = pf.num_unique;
    if (pf.trace_rows.n != nu * 7 * 8 || pf.constraint_rows.n != nu * 8 * de)
        return "ProofDeserializationError(\"query count\")";
    auto draw = [&](Coin& coin, E2& out) {
        u64 v[2] = {0, 0};
        if (!coin.draw_e(v, de)) return false;
        out = E2{v[0], v[1]};
        return true;
    };

    // ---- transcript
    u64 seed[20];
    context_elements(n, o, seed);
    memcpy(seed + 8, air.pub, 12 * 8);
    Coin coin;
    coin.init(seed, 20);
    coin.reseed(pf.com[0]);
    E2 alpha[7], bc[8];
    for (auto& x : alpha)
        if (!draw(coin, x)) return "RandomCoinError";
    for (auto& x : bc)
        if (!draw(coin, x)) return "RandomCoinError";
    coin.reseed(pf.com[1]);
    E2 z;
    if (!draw(coin, z)) return "RandomCoinError";
    const u64 g = gl_root((unsigned)pf.logn), g_last = gl_pow(g, n - 1);
    const E2 zg = e2_mulb(z, g);
    E2 ood[14];
    for (int k = 0; k < 14; k++) ood[k] = elem_e(pf.ood, k, de);
    const E2 hz = elem_e(pf.hz, 0, de);

    // ---- OOD consistency: H(z) == sum alpha_i r_i(z) Z_t(z)^-1 + boundary terms
    {
        E2 cur[7], nxt[7], rr[7];
        for (int c = 0; c < 7; c++) {
            cur[c] = ood[2 * c];
            nxt[c] = ood[2 * c + 1];
        }
        air_transition(air, cur, nxt, rr);
        E2 t{0, 0};
        for (int c = 0; c < 7; c++) t = e2_add(t, e2_mul(alpha[c], rr[c]));
        const E2 zn1 = e2_sub(e2_pow(z, n), e2(1)), z1 = e2_sub(z, e2(1)), zl = e2_sub(z, e2(g_last));
        if (e2_eq(zn1, e2(0)) || e2_eq(z1, e2(0)) || e2_eq(zl, e2(0))) return "InconsistentOodConstraintEvaluations";
        E2 ev = e2_mul(e2_mul(t, zl), e2_inv(zn1));
        const u64 v0[7] = {air.pub[0], air.pub[1], air.pub[2], air.pub[3], 0, air.nullifier, air.commitment};
        E2 b0{0, 0};
        for (int c = 0; c < 7; c++) b0 = e2_add(b0, e2_mul(bc[c], e2_sub(cur[c], e2(v0[c]))));
        const E2 b1 = e2_mul(bc[7], e2_sub(cur[4], e2(3)));
        ev = e2_add(ev, e2_mul(b0, e2_inv(z1)));
        ev = e2_add(ev, e2_mul(b1, e2_inv(zl)));
        if (!e2_eq(ev, hz)) return "InconsistentOodConstraintEvaluations";
    }
    {
        std::vector<u64> raw(15 * de);
        memcpy(raw.data(), pf.ood.p, 14 * 8 * de);
        memcpy(raw.data() + 14 * de, pf.hz.p, 8 * de);
        coin.reseed(hash_elements(raw.data(), 14 * de));
        coin.reseed(hash_elements(raw.data() + 14 * de, de));
    }
    E2 dc[7], gam;
    for (auto& x : dc)
        if (!draw(coin, x)) return "RandomCoinError";
    if (!draw(coin, gam)) return "RandomCoinError";
    std::vector<E2> falpha(nl);
    for (unsigned l = 0; l <= nl; l++) {
        coin.reseed(pf.com[2 + l]);
        E2 a;
        if (!draw(coin, a)) return "RandomCoinError";
        if (l < nl) falpha[l] = a;
    }
    // ---- proof of work + query positions
    {
        Digest h = merge_with_int(coin.seed, pf.nonce);
        if (tz64((u64)h.w[0] | ((u64)h.w[1] << 32)) < o.grind) return "QuerySeedProofOfWorkVerificationFailed";
    }
    coin.reseed_int(pf.nonce);
    std::vector<u64> pos(o.q);
    for (auto& x : pos) {
        Digest h = coin.next();
        x = ((u64)h.w[0] | ((u64)h.w[1] << 32)) & (N - 1);
    }
    std::sort(pos.begin(), pos.end());
    pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
    if (pos.size() != nu) return "ProofDeserializationError(\"number of unique queries\")";

    st.de = de;
    st.n = n;
    st.N = N;
    st.beta = beta;
    st.nl = nl;
    st.pos = std::move(pos);
    st.z = z;
    st.zg = zg;
    st.hz = hz;
    for (int k = 0; k < 14; k++) st.ood[k] = ood[k];
    for (int k = 0; k < 7; k++) st.dc[k] = dc[k];
    st.gam = gam;
    st.falpha = std::move(falpha);
    return "";
}

std::string verify_queries_host(const VState& st) {
    const ParsedProof& pf = st.pf;
    const int de = st.de;
    const u64 N = st.N, beta = st.beta, nu = pf.num_unique, depthN = ilog2(N);
    const unsigned nl = st.nl;
    const std::vector<u64>& pos = st.pos;
    const E2 z = st.z, zg = st.zg, hz = st.hz, gam = st.gam;
    const E2* ood = st.ood;
    const E2* dc = st.dc;
    const std::vector<E2>& falpha = st.falpha;
    // ---- trace / constraint openings
    std::vector<Digest> leaves(nu);
    Digest root;
    for (u64 i = 0; i < nu; i++) leaves[i] = leaf_hash(pf.trace_rows.p + i * 56, 56);
    if (!batch_root(pos, leaves, pf.trace_paths, N, root) || !same(root, pf.com[0]))
        return "TraceQueryDoesNotMatchCommitment";
    for (u64 i = 0; i < nu; i++) leaves[i] = leaf_hash(pf.constraint_rows.p + i * 8 * de, 8 * de);
    if (!batch_root(pos, leaves, pf.constraint_paths, N, root) || !same(root, pf.com[1]))
        return "ConstraintQueryDoesNotMatchCommitment";

    // ---- DEEP composition at the query points
    std::vector<E2> ev(nu);
    const u64 wN = gl_root((unsigned)depthN);
    for (u64 i = 0; i < nu; i++) {
        const E2 x = e2(gl_mul(GEN, gl_pow(wN, pos[i])));
        E2 s1{0, 0}, s2{0, 0};
        for (int c = 0; c < 7; c++) {
            const E2 tx = e2(pf.trace_rows.elem(i * 7 + c));
            s1 = e2_add(s1, e2_mul(dc[c], e2_sub(tx, ood[2 * c])));
            s2 = e2_add(s2, e2_mul(dc[c], e2_sub(tx, ood[2 * c + 1])));
        }
        const E2 izx = e2_inv(e2_sub(x, z)), izgx = e2_inv(e2_sub(x, zg));
        E2 d = e2_add(e2_mul(s1, izx), e2_mul(s2, izgx));
        d = e2_add(d, e2_mul(e2_mul(gam, e2_sub(elem_e(pf.constraint_rows, i, de), hz)), izx));
        ev[i] = d;
    }

    // ---- FRI: each layer's openings, folding consistency, remainder
    std::vector<u64> cur = pos;
    u64 D = N;
    for (unsigned l = 0; l < nl; l++) {
        const u64 rows = D / 8;
        std::vector<u64> fp = fold_positions(cur, rows);
        const Span& vals = pf.fri_vals[l];
        if (vals.n != fp.size() * 64 * de) return "FriVerificationFailed(InvalidLayerCommitment)";
        std::vector<Digest> lv(fp.size());
        for (size_t i = 0; i < fp.size(); i++) lv[i] = leaf_hash(vals.p + i * 64 * de, 64 * de);
        if (!batch_root(fp, lv, pf.fri_paths[l], rows, root) || !same(root, pf.com[2 + l]))
            return "FriVerificationFailed(LayerCommitmentMismatch)";
        for (size_t i = 0; i < cur.size(); i++) {
            const u64 ri = cur[i] & (rows - 1), k = cur[i] / rows;
            const size_t at = std::find(fp.begin(), fp.end(), ri) - fp.begin();
            if (!e2_eq(elem_e(vals, at * 8 + k, de), ev[i])) return "FriVerificationFailed(InvalidLayerFolding)";
        }
        const u64 wD = gl_root(ilog2(D));
        std::vector<E2> nev(fp.size());
        for (size_t i = 0; i < fp.size(); i++) {
            E2 v[8];
            for (int k = 0; k < 8; k++) v[k] = elem_e(vals, i * 8 + k, de);
            nev[i] = fold_row(v, gl_mul(GEN, gl_pow(wD, fp[i])), falpha[l]);
        }
        cur.swap(fp);
        ev.swap(nev);
        D = rows;
    }
    const u64 rl = pf.fri_rem.n / (8 * de);
    if (rl == 0 || rl != D / beta) return "FriVerificationFailed(InvalidRemainderFolding)";
    std::vector<u64> raw(rl * de);
    memcpy(raw.data(), pf.fri_rem.p, rl * 8 * de);
    if (!same(hash_elements(raw.data(), rl * de), pf.com[2 + nl]))
        return "FriVerificationFailed(RemainderCommitmentMismatch)";
    const u64 wD = gl_root(ilog2(D));
    for (size_t i = 0; i < cur.size(); i++) {
        const E2 x = e2(gl_mul(GEN, gl_pow(wD, cur[i])));
        E2 r{0, 0};
        for (u64 k = rl; k-- > 0;) r = e2_add(e2_mul(r, x), elem_e(pf.fri_rem, k, de));
        if (!e2_eq(r, ev[i])) return "FriVerificationFailed(InvalidRemainderFolding)";
    }
    return "";
}

static std::string verify_proof(const uint8_t* bytes, size_t len, const AirConst& air, const Opts& acceptable) {
    VState st;
    std::string e = verify_transcript(bytes, len, air, acceptable, st);
    return e.empty() ? verify_queries_host(st) : e;
}

// ------------------------------------------------------------------ batched GPU verification plan
bool plan_proof(const VState& st, size_t blob_off, VerifyPlan& plan, std::string& err) {
    const ParsedProof& pf = st.pf;
    const int de = st.de;
    const u64 N = st.N, nu = pf.num_unique;
    const unsigned nl = st.nl;
    plan.trees.clear();
    plan.tleaves.clear();
    plan.vecs.clear();
    plan.fqueries.clear();
    if (nl > (unsigned)VMAXL) {
        err = "ProofDeserializationError(\"too many FRI layers\")";
        return false;
    }
    auto off = [&](const uint8_t* p) { return (u64)blob_off + (u64)(p - pf.base); };
    // FRI position lists (first-occurrence order, the order of the opened rows) and the structural
    // checks the host verifier makes before it opens anything
    thread_local std::vector<std::vector<u64>> fps;
    fps.resize(nl);
    {
        const std::vector<u64>* cur = &st.pos;
        u64 D = N;
        for (unsigned l = 0; l < nl; l++) {
            const u64 rows = D / 8;
            fps[l] = fold_positions(*cur, rows);
            if (pf.fri_vals[l].n != fps[l].size() * 64 * de) {
                err = "FriVerificationFailed(InvalidLayerCommitment)";
                return false;
            }
            cur = &fps[l];
            D = rows;
        }
        const u64 rl = pf.fri_rem.n / (8 * de);
        if (rl == 0 || rl != D / st.beta) {
            err = "FriVerificationFailed(InvalidRemainderFolding)";
            return false;
        }
    }
    // one VTree per batch opening: the opened rows sorted by leaf index, the node vectors as the
    // proof holds them; the device checks that they fit the opening (BatchMerkleProof::get_root)
    auto add_tree = [&](const u64* idx, size_t cnt, const Paths& paths, unsigned depth, const uint8_t* row0,
                        size_t stride, uint32_t words, unsigned com, uint32_t bit) {
        VTree t{};
        t.root_off = off(pf.com_p + 32 * com);
        t.leaf0 = (uint32_t)plan.tleaves.size();
        t.nidx = (uint32_t)cnt;
        t.vec0 = (uint32_t)plan.vecs.size();
        t.nvec = (uint32_t)paths.ptr.size();
        t.words = words;
        t.depth = depth;
        t.bit = bit;
        const size_t l0 = plan.tleaves.size();
        for (size_t i = 0; i < cnt; i++) plan.tleaves.push_back(VTreeLeaf{idx[i], off(row0 + i * stride)});
        std::sort(plan.tleaves.begin() + l0, plan.tleaves.end(),
                  [](const VTreeLeaf& x, const VTreeLeaf& y) { return x.index < y.index; });
        for (size_t v = 0; v < paths.ptr.size(); v++) plan.vecs.push_back(VVec{off(paths.ptr[v]), paths.cnt[v], 0});
        plan.trees.push_back(t);
    };
    const unsigned depthN = ilog2(N);
    add_tree(st.pos.data(), nu, pf.trace_paths, depthN, pf.trace_rows.p, 56, 7, 0, VF_TRACE);
    add_tree(st.pos.data(), nu, pf.constraint_paths, depthN, pf.constraint_rows.p, 8 * de, (uint32_t)de, 1,
             VF_CONSTRAINT);
    for (unsigned l = 0; l < nl; l++)
        add_tree(fps[l].data(), fps[l].size(), pf.fri_paths[l], depthN - 3 * (l + 1), pf.fri_vals[l].p, 64 * de,
                 (uint32_t)(8 * de), 2 + l, 1u << (VF_LAYER_COMMIT + l));
    // field checks
    VFieldProof& F = plan.fproof;
    F = VFieldProof{};
    F.z = st.z;
    F.zg = st.zg;
    F.hz = st.hz;
    F.gam = st.gam;
    for (int k = 0; k < 7; k++) F.dc[k] = st.dc[k];
    for (int k = 0; k < 14; k++) F.ood[k] = st.ood[k];
    for (unsigned l = 0; l < nl; l++) F.falpha[l] = st.falpha[l];
    F.rem_off = off(pf.fri_rem.p);
    F.rem_len = (uint32_t)(pf.fri_rem.n / (8 * de));
    F.nl = nl;
    F.de = (uint32_t)de;
    F.logN = depthN;
    for (u64 i = 0; i < nu; i++) {
        VFieldQuery Q{};
        Q.pos = st.pos[i];
        Q.trace_off = off(pf.trace_rows.p + i * 56);
        Q.cons_off = off(pf.constraint_rows.p + i * 8 * de);
        u64 p = st.pos[i], D = N;
        for (unsigned l = 0; l < nl; l++) {
            const u64 rows = D / 8, r = p & (rows - 1);
            const size_t at = std::find(fps[l].begin(), fps[l].end(), r) - fps[l].begin();
            Q.row_off[l] = off(pf.fri_vals[l].p + at * 64 * de);
            p = r;
            D = rows;
        }
        plan.fqueries.push_back(Q);
    }
    return true;
}

std::string finish_proof(const VState& st, uint32_t flags) {
    const ParsedProof& pf = st.pf;
    if (flags & VF_TRACE) return "TraceQueryDoesNotMatchCommitment";
    if (flags & VF_CONSTRAINT) return "ConstraintQueryDoesNotMatchCommitment";
    for (unsigned l = 0; l < st.nl; l++) {
        if (flags & (1u << (VF_LAYER_COMMIT + l))) return "FriVerificationFailed(LayerCommitmentMismatch)";
        if (flags & (1u << l)) return "FriVerificationFailed(InvalidLayerFolding)";
    }
    const u64 rl = pf.fri_rem.n / (8 * st.de);
    std::vector<u64> raw(rl * st.de);
    memcpy(raw.data(), pf.fri_rem.p, rl * 8 * st.de);
    if (!same(hash_elements(raw.data(), rl * st.de), pf.com[2 + st.nl]))
        return "FriVerificationFailed(RemainderCommitmentMismatch)";
    if (flags & VF_REMAINDER) return "FriVerificationFailed(InvalidRemainderFolding)";
    return "";
}

AirConst air_of(const xfg_air_consts* a) {
    AirConst c;
    memset(&c, 0, sizeof c);
    memcpy(c.pub, a->pub_inputs, sizeof a->pub_inputs);
    c.nullifier = a->nullifier;
    c.commitment = a->commitment;
    return c;
}
static void put_err(const std::string& e, char* buf, size_t len) {
    if (!buf || !len) return;
    size_t k = std::min(len - 1, e.size());
    memcpy(buf, e.data(), k);
    buf[k] = 0;
}

}  // namespace xfg

using namespace xfg;

extern "C" {

int xfg_proof_parse(const uint8_t* proof, size_t len, xfg_proof_info* info, char* err, size_t err_len) {
    if (!proof || !info) return XFG_INVALID_ARGUMENT;
    ParsedProof pf;
    std::string e = parse_proof(proof, len, pf);
    put_err(e, err, err_len);
    if (!e.empty()) return XFG_VERIFY_FAILED;
    memset(info, 0, sizeof *info);
    info->trace_width = (uint32_t)pf.width;
    info->trace_length = 1ULL << pf.logn;
    info->options.num_queries = (uint32_t)pf.o.q;
    info->options.blowup_factor = (uint32_t)pf.o.beta;
    info->options.grinding_factor = (uint32_t)pf.o.grind;
    info->options.field_extension = (uint32_t)pf.o.ext;
    info->options.fri_folding_factor = (uint32_t)pf.o.fold;
    info->options.fri_remainder_max_degree = (uint32_t)pf.o.remdeg;
    info->num_unique_queries = (uint32_t)pf.num_unique;
    info->num_fri_layers = (uint32_t)pf.fri_vals.size();
    const size_t de = (size_t)pf.o.ext;  // coordinates per E element (parse_proof: 1..3)
    info->remainder_len = (uint32_t)(pf.fri_rem.n / (8 * de));
    info->pow_nonce = pf.nonce;
    info->size = pf.size;
    for (size_t i = 0; i < 2 && i < pf.com.size(); i++) memcpy(i ? info->constraint_root : info->trace_root, pf.com[i].w, 32);
    // with an extension: first coordinates; a frame narrower than 7 columns leaves the rest 0, and a
    // frame whose contents do not parse (which from_bytes does not look at) leaves all of it 0
    if (parse_contents(pf).empty()) {
        const size_t frame = pf.ood.n / (8 * de);
        for (size_t k = 0; k < 14 && k < frame; k++) info->ood_trace[k] = pf.ood.elem(k * de);
        info->ood_composition = pf.hz.elem(0);
    }
    return XFG_OK;
}

int xfg_verify(const uint8_t* proof, size_t len, const xfg_air_consts* air, const xfg_options* acceptable, char* err,
               size_t err_len) {
    if (!proof || !air || !acceptable) return XFG_INVALID_ARGUMENT;
    std::string e;
    try {
        e = verify_proof(proof, len, air_of(air), to_opts(acceptable));
    } catch (const std::exception& x) {
        e = std::string("ProofDeserializationError(\"") + x.what() + "\")";
    }
    put_err(e, err, err_len);
    return e.empty() ? XFG_OK : XFG_VERIFY_FAILED;
}

int xfg_selftest_blake3(const uint8_t* in, size_t len, uint8_t out[32]) {
    if ((!in && len) || !out) return XFG_INVALID_ARGUMENT;
    Digest d = blake3_bytes(in, len);
    digest_bytes(d, out);
    return XFG_OK;
}

int xfg_verify_batch(uint32_t count, const uint8_t* const* proofs, const size_t* lens, const xfg_air_consts* airs,
                     const xfg_options* acceptable, int* results, uint32_t threads) {
    if (!proofs || !lens || !airs || !acceptable || !results) return XFG_INVALID_ARGUMENT;
    unsigned nt = threads ? threads : std::max(1u, std::thread::hardware_concurrency());
    nt = std::min<unsigned>(nt, std::max<uint32_t>(1, count));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            for (uint32_t i = t; i < count; i += nt)
                results[i] = proofs[i] ? xfg_verify(proofs[i], lens[i], &airs[i], acceptable, nullptr, 0)
                                       : XFG_INVALID_ARGUMENT;
        });
    for (auto& x : th) x.join();
    return XFG_OK;
}

}  // extern "C"
