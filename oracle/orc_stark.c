/*
 * ORACLE / TEST INFRASTRUCTURE ONLY (see oracle.h for the scope and parity status).
 *
 * Single-threaded C restatement of the XFG burn-proof STARK prover + verifier:
 *   burn AIR (reference src/burn_mint_air.rs) + marshalling (src/burn_mint_prover.rs), and the
 *   Winterfell 0.8.3 pipeline that `air.prove(trace)` runs (src/burn_mint_prover.rs:124-126).
 * Steps marked RECALLED restate Winterfell 0.8 behaviour from its published design (the crate
 * is not vendored in /root/reference); they are this project's definition
 * of the proof format and are what the GPU path must reproduce bit for bit.
 *
 * Arithmetic here is deliberately the plain textbook form (radix-2 NTT over a zero-padded
 * domain, Horner evaluation, naive 8-point interpolation for FRI folds) so that it shares no
 * structure with the HIP implementation it checks.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle.h"
#include "orc_prims.h"

/* per-thread stage timers (orc_prove_batch): CPU milliseconds per prover stage, ORC_NSTAGE slots */
static _Thread_local double* t_stage;
static _Thread_local double t_mark;
static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
#define STAGE(i)                                   \
    do {                                           \
        if (t_stage) {                             \
            const double t_ = now_ms();            \
            t_stage[i] += t_ - t_mark;             \
            t_mark = t_;                           \
        }                                          \
    } while (0)

/* ============================================================ exported primitive wrappers */
void orc_blake3_bytes(const uint8_t* in, size_t len, uint8_t out[32]) { orc_blake3(in, len, out); }
void orc_keccak256_bytes(const uint8_t* in, size_t len, uint8_t out[32]) { orc_keccak256(in, len, out); }
void orc_sha3_256_bytes(const uint8_t* in, size_t len, uint8_t out[32]) { orc_keccak_sponge(in, len, 0x06, out); }
uint64_t orc_field_mul(uint64_t a, uint64_t b) { return orc_mul(a, b); }
uint64_t orc_field_root(uint32_t k) { return orc_root(k); }

static void put_le64(uint8_t* d, uint64_t v) { for (int i = 0; i < 8; i++) d[i] = (uint8_t)(v >> (8 * i)); }
static uint64_t get_le64(const uint8_t* s) { uint64_t v = 0; for (int i = 0; i < 8; i++) v |= (uint64_t)s[i] << (8 * i); return v; }
static unsigned ilog2u(uint64_t x) { unsigned r = 0; while ((1ULL << r) < x) r++; return r; }
static int is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

/* ============================================================ NTT (winter-math fft, restated) */
static void ntt_inplace(uint64_t* a, uint64_t n, uint64_t root) {
    /* natural order in -> natural order out: a_k <- sum_j a_j root^(jk) */
    for (uint64_t i = 1, j = 0; i < n; i++) {
        uint64_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { uint64_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
    for (uint64_t len = 2; len <= n; len <<= 1) {
        uint64_t wl = orc_pow(root, n / len);
        for (uint64_t i = 0; i < n; i += len) {
            uint64_t w = 1;
            for (uint64_t k = 0; k < len / 2; k++) {
                uint64_t u = a[i + k], v = orc_mul(a[i + k + len / 2], w);
                a[i + k] = orc_add(u, v);
                a[i + k + len / 2] = orc_sub(u, v);
                w = orc_mul(w, wl);
            }
        }
    }
}
/* fft::interpolate_poly_with_offset: evaluations at offset*w_n^i -> coefficients */
void orc_interpolate(uint64_t* vals, uint64_t n, uint64_t offset) {
    ntt_inplace(vals, n, orc_inv(orc_root(ilog2u(n))));
    uint64_t ninv = orc_inv(n % ORC_P), oinv = orc_inv(offset), s = ninv;
    for (uint64_t j = 0; j < n; j++) { vals[j] = orc_mul(vals[j], s); s = orc_mul(s, oinv); }
}
/* fft::evaluate_poly_with_offset: coefficients -> values at offset*w_N^k, k natural, N = n*blowup */
void orc_evaluate_lde(const uint64_t* coef, uint64_t n, uint64_t blowup, uint64_t offset, uint64_t* out) {
    uint64_t N = n * blowup, s = 1;
    memset(out, 0, N * sizeof(uint64_t));
    for (uint64_t j = 0; j < n; j++) { out[j] = orc_mul(coef[j], s); s = orc_mul(s, offset); }
    ntt_inplace(out, N, orc_root(ilog2u(N)));
}
static uint64_t horner(const uint64_t* c, uint64_t n, uint64_t x) {
    uint64_t r = 0;
    for (uint64_t j = n; j-- > 0;) r = orc_add(orc_mul(r, x), c[j]);
    return r;
}
/* polynom::syn_div_in_place(a, 1, b): quotient of a(x)/(x-b) in place, top slot zeroed */
static void syn_div(uint64_t* a, uint64_t n, uint64_t b) {
    uint64_t c = 0;
    for (uint64_t j = n; j-- > 0;) {
        uint64_t v = orc_add(a[j], orc_mul(b, c));
        a[j] = c;
        c = v;
    }
}

/* ============================================================ Merkle tree (winter-crypto) */
typedef uint8_t dg[32];
static void hash_elems(const uint64_t* e, size_t cnt, uint8_t out[32]) {
    /* Blake3_256::hash_elements: BLAKE3 over canonical LE encodings (f64 is non-canonical
     * internally, so winter-crypto serialises through ByteWriter -> same bytes) */
    uint8_t stackbuf[512] = {0};
    uint8_t* buf = cnt * 8 <= sizeof stackbuf ? stackbuf : (uint8_t*)malloc(cnt * 8);
    for (size_t i = 0; i < cnt; i++) put_le64(buf + 8 * i, e[i]);
    orc_blake3(buf, cnt * 8, out);
    if (buf != stackbuf) free(buf);
}
static void merge2(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    uint8_t buf[64];
    memcpy(buf, a, 32); memcpy(buf + 32, b, 32);
    orc_blake3(buf, 64, out);
}
static void merge_int(const uint8_t a[32], uint64_t v, uint8_t out[32]) {
    uint8_t buf[40];
    memcpy(buf, a, 32); put_le64(buf + 32, v);
    orc_blake3(buf, 40, out);
}
typedef struct { uint64_t L; dg* nodes; } mtree; /* nodes[1]=root, nodes[L+i]=leaf i */
static void mtree_build(mtree* t, dg* leaves, uint64_t L) {
    t->L = L;
    t->nodes = (dg*)malloc(2 * L * sizeof(dg));
    memcpy(t->nodes + L, leaves, L * sizeof(dg));
    for (uint64_t i = L - 1; i >= 1; i--) merge2(t->nodes[2 * i], t->nodes[2 * i + 1], t->nodes[i]);
    memset(t->nodes[0], 0, 32);
}
static void mtree_free(mtree* t) { free(t->nodes); t->nodes = NULL; }

/* growable byte buffer (winter-utils ByteWriter) */
typedef struct { uint8_t* b; size_t n, cap; } bbuf;
static void bb_put(bbuf* w, const void* p, size_t k) {
    if (w->n + k > w->cap) { w->cap = (w->n + k) * 2 + 64; w->b = (uint8_t*)realloc(w->b, w->cap); }
    memcpy(w->b + w->n, p, k); w->n += k;
}
static void bb_u8(bbuf* w, uint8_t v) { bb_put(w, &v, 1); }
static void bb_u16(bbuf* w, uint16_t v) { uint8_t d[2] = {(uint8_t)v, (uint8_t)(v >> 8)}; bb_put(w, d, 2); }
static void bb_u32(bbuf* w, uint32_t v) { uint8_t d[4]; for (int i = 0; i < 4; i++) d[i] = (uint8_t)(v >> (8 * i)); bb_put(w, d, 4); }
static void bb_u64(bbuf* w, uint64_t v) { uint8_t d[8]; put_le64(d, v); bb_put(w, d, 8); }

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}
/* MerkleTree::prove_batch + BatchMerkleProof::serialize_nodes (RECALLED, winter-crypto 0.8.3):
 * leaf pairs are taken in ascending normalised order; node vector i collects the siblings met by
 * the i-th entry of the current level's index list (the list shrinks as siblings merge). */
static void mtree_prove_serialize(const mtree* t, const uint64_t* idx, uint64_t k, bbuf* out) {
    uint64_t L = t->L, depth = ilog2u(L);
    uint64_t* norm = (uint64_t*)malloc(k * sizeof(uint64_t));
    uint64_t m = 0;
    for (uint64_t i = 0; i < k; i++) norm[m++] = idx[i] & ~1ULL;
    qsort(norm, m, sizeof(uint64_t), cmp_u64);
    uint64_t u = 0;
    for (uint64_t i = 0; i < m; i++) if (u == 0 || norm[u - 1] != norm[i]) norm[u++] = norm[i];
    m = u;
    /* node vectors: nv[i] holds up to depth digests */
    dg* nv = (dg*)malloc(m * depth * sizeof(dg));
    uint64_t* nvc = (uint64_t*)calloc(m, sizeof(uint64_t));
    uint64_t* cur = (uint64_t*)malloc(m * sizeof(uint64_t));
    uint64_t* nxt = (uint64_t*)malloc(m * sizeof(uint64_t));
    for (uint64_t i = 0; i < m; i++) {
        for (uint64_t leaf = norm[i]; leaf < norm[i] + 2; leaf++) {
            int requested = 0;
            for (uint64_t q = 0; q < k; q++) if (idx[q] == leaf) { requested = 1; break; }
            if (!requested) memcpy(nv[i * depth + nvc[i]++], t->nodes[L + leaf], 32);
        }
        cur[i] = (norm[i] + L) >> 1;
    }
    uint64_t cn = m;
    for (uint64_t lvl = 1; lvl < depth; lvl++) {
        uint64_t nn = 0;
        for (uint64_t i = 0; i < cn; i++) {
            uint64_t sib = cur[i] ^ 1;
            if (i + 1 < cn && cur[i + 1] == sib) i++;
            else memcpy(nv[i * depth + nvc[i]++], t->nodes[sib], 32);
            nxt[nn++] = sib >> 1;
        }
        uint64_t* tmp = cur; cur = nxt; nxt = tmp; cn = nn;
    }
    bb_u8(out, (uint8_t)m);
    for (uint64_t i = 0; i < m; i++) {
        bb_u8(out, (uint8_t)nvc[i]);
        bb_put(out, nv[i * depth], nvc[i] * 32);
    }
    free(norm); free(nv); free(nvc); free(cur); free(nxt);
}

/* ============================================================ DefaultRandomCoin<Blake3_256> */
typedef struct { uint8_t seed[32]; uint64_t counter; } coin_t;
static void coin_init(coin_t* c, const uint64_t* e, size_t cnt) { hash_elems(e, cnt, c->seed); c->counter = 0; }
static void coin_reseed(coin_t* c, const uint8_t d[32]) { uint8_t s[32]; merge2(c->seed, d, s); memcpy(c->seed, s, 32); c->counter = 0; }
static void coin_reseed_int(coin_t* c, uint64_t v) { uint8_t s[32]; merge_int(c->seed, v, s); memcpy(c->seed, s, 32); c->counter = 0; }
static void coin_next(coin_t* c, uint8_t out[32]) { c->counter++; merge_int(c->seed, c->counter, out); }
static int coin_draw(coin_t* c, uint64_t* out) {
    for (int i = 0; i < 1000; i++) {
        uint8_t v[32];
        coin_next(c, v);
        uint64_t x = get_le64(v);
        if (x < ORC_P) { *out = x; return 0; }
    }
    return -1;
}
static unsigned tz64(uint64_t x) { if (!x) return 64; unsigned r = 0; while (!(x & 1)) { x >>= 1; r++; } return r; }

/* ============================================================ burn AIR */
#define STANDARD_BURN 8000000ULL
#define LARGE_BURN 8000000000ULL
enum { PI_BURN, PI_MINT, PI_TXN, PI_RH, PI_STATE, PI_TX0, PI_TX1, PI_TX2, PI_TX3, PI_NET, PI_CHAIN, PI_VER };

/* src/burn_mint_air.rs:124-133 compute_nullifier, :157-170 compute_recipient_hash,
 * :174-202 compute_commitment */
void orc_air_constants(const uint64_t pub[12], uint64_t secret, uint64_t* nullifier, uint8_t rfull[32],
                       uint64_t* commitment) {
    uint8_t buf[200], h[32];
    size_t k = 0;
    put_le64(buf, secret); k = 8;
    memcpy(buf + k, "nullifier", 9); k += 9;
    put_le64(buf + k, pub[PI_BURN]); k += 8;
    orc_keccak256(buf, k, h);
    *nullifier = (uint64_t)h[0] | ((uint64_t)h[1] << 8) | ((uint64_t)h[2] << 16) | ((uint64_t)h[3] << 24);

    uint8_t rf[32];
    k = 0;
    put_le64(buf, pub[PI_RH]); k = 8;
    memcpy(buf + k, "ethereum-recipient", 18); k += 18;
    memcpy(buf + k, "fuego-to-heat-bridge", 20); k += 20;
    orc_keccak256(buf, k, rf);
    if (rfull) memcpy(rfull, rf, 32);

    k = 0;
    put_le64(buf + k, secret); k += 8;
    put_le64(buf + k, pub[PI_BURN]); k += 8;
    put_le64(buf + k, pub[PI_MINT]); k += 8;
    for (int i = 0; i < 4; i++) { put_le64(buf + k, pub[PI_TX0 + i]); k += 8; }
    memcpy(buf + k, rf, 32); k += 32;
    put_le64(buf + k, pub[PI_NET]); k += 8;
    put_le64(buf + k, pub[PI_CHAIN]); k += 8;
    put_le64(buf + k, pub[PI_VER]); k += 8;
    memcpy(buf + k, "heat-commitment-v1", 18); k += 18;
    orc_keccak256(buf, k, h);
    *commitment = (uint64_t)h[0] | ((uint64_t)h[1] << 8) | ((uint64_t)h[2] << 16) | ((uint64_t)h[3] << 24);
}

/* src/burn_mint_prover.rs:62-118 (marshalling), :132-180 (validate_inputs), :195-208, :211-221 */
int orc_burn_air_from_inputs(uint64_t burn, uint64_t mint, const uint8_t tx[32], const uint8_t* recipient,
                             size_t rlen, const uint8_t* secret, size_t slen, uint32_t network_id,
                             uint32_t target_chain_id, uint32_t commitment_version, orc_air* out) {
    uint64_t legacy = get_le64(tx);
    if (burn != STANDARD_BURN && burn != LARGE_BURN) return ORC_INVALID_BURN_AMOUNT;
    if (mint != burn) return ORC_MINT_MISMATCH;
    if (legacy == 0) return ORC_ZERO_TX_HASH;
    if (rlen != 20) return ORC_BAD_RECIPIENT_LEN;
    /* reference: <4 -> error, 4..7 -> slice panic (:203-204); the contract maps both to SHORT_SECRET */
    if (slen < 8) return ORC_SHORT_SECRET;
    uint64_t secret_el = (uint64_t)secret[0] | ((uint64_t)secret[1] << 8) | ((uint64_t)secret[2] << 16) |
                         ((uint64_t)secret[3] << 24);
    uint8_t buf[64], h[32];
    memcpy(buf, recipient, 20);
    memcpy(buf + 20, "recipient", 9);
    orc_keccak256(buf, 29, h);
    uint64_t rh = (uint64_t)h[0] | ((uint64_t)h[1] << 8) | ((uint64_t)h[2] << 16) | ((uint64_t)h[3] << 24);
    uint64_t* p = out->pub;
    p[PI_BURN] = (uint32_t)burn;
    p[PI_MINT] = (uint32_t)mint;
    p[PI_TXN] = (uint32_t)legacy;
    p[PI_RH] = rh;
    p[PI_STATE] = 0;
    for (int i = 0; i < 4; i++)
        p[PI_TX0 + i] = (uint64_t)tx[4 * i] | ((uint64_t)tx[4 * i + 1] << 8) | ((uint64_t)tx[4 * i + 2] << 16) |
                        ((uint64_t)tx[4 * i + 3] << 24);
    p[PI_NET] = network_id;
    p[PI_CHAIN] = target_chain_id;
    p[PI_VER] = commitment_version;
    out->secret = secret_el;
    orc_air_constants(p, secret_el, &out->nullifier, NULL, &out->commitment);
    return ORC_OK;
}

/* src/burn_mint_air.rs:442-476 build_trace, made length-generic */
void orc_build_trace(const orc_air* air, uint64_t n, uint64_t* tr) {
    for (uint64_t s = 0; s < n; s++) {
        tr[0 * n + s] = air->pub[PI_BURN];
        tr[1 * n + s] = air->pub[PI_MINT];
        tr[2 * n + s] = air->pub[PI_TXN];
        tr[3 * n + s] = air->pub[PI_RH];
        tr[4 * n + s] = (4 * s) / n;
        tr[5 * n + s] = air->nullifier;
        tr[6 * n + s] = air->commitment;
    }
}

/* src/burn_mint_air.rs:335-378 evaluate_transition (7 constraints, corrected AIR A.2) */
static void air_transition(const orc_air* air, const uint64_t cur[7], const uint64_t nxt[7], int faithful,
                           uint64_t r[7]) {
    uint64_t nullifier = air->nullifier, commitment = air->commitment;
    if (faithful) { /* the reference recomputes both Keccak constants on every call (:264, :376) */
        orc_air_constants(air->pub, air->secret, &nullifier, NULL, &commitment); /* 3 Keccak-256 */
    }
    uint64_t std_burn = STANDARD_BURN, large = orc_mul(STANDARD_BURN, 1000); /* :207-219 in-field */
    r[0] = orc_mul(orc_sub(cur[0], std_burn), orc_sub(cur[0], large));
    r[1] = orc_sub(cur[1], cur[0]);
    r[2] = orc_sub(cur[2], (uint32_t)air->pub[PI_TXN]);
    r[3] = orc_sub(cur[3], (uint32_t)air->pub[PI_RH]);
    uint64_t d = orc_sub(nxt[4], cur[4]);
    r[4] = orc_mul(d, orc_sub(d, 1));
    r[5] = orc_sub(cur[5], nullifier);
    r[6] = orc_sub(cur[6], commitment);
}
void orc_eval_transition(const orc_air* air, const uint64_t cur[7], const uint64_t nxt[7], uint64_t r[7]) {
    air_transition(air, cur, nxt, 0, r);
}
/* src/burn_mint_air.rs:380-395 get_assertions: 8 single assertions, final step n-1 (A.3);
 * already in Winterfell's (stride, first_step, column) order. */
static void air_assertions(const orc_air* air, uint64_t n, uint64_t col[8], uint64_t step[8], uint64_t val[8]) {
    const uint64_t v0[7] = {air->pub[PI_BURN], air->pub[PI_MINT], air->pub[PI_TXN], air->pub[PI_RH], 0,
                            air->nullifier, air->commitment};
    for (int i = 0; i < 7; i++) { col[i] = (uint64_t)i; step[i] = 0; val[i] = v0[i]; }
    col[7] = 4; step[7] = n - 1; val[7] = 3;
}

/* ============================================================ proof options / context */
#define W 7
#define NUM_ASSERT 8
#define CE_BLOWUP 2 /* max(next_pow2(declared degree 1), MIN_BLOWUP_FACTOR 2) -- RECALLED */
static int check_options(uint64_t n, const orc_options* o) {
    if (!is_pow2(n) || n < 8 || n > (1ULL << 26)) return -1;
    if (!is_pow2(o->blowup) || o->blowup < CE_BLOWUP || o->blowup > 128) return -1;
    if (o->num_queries < 1 || o->num_queries > 255) return -1;
    if (o->grinding > 32) return -1;
    if (o->field_extension != 1 && o->field_extension != 2) return -1; /* None or Quadratic */
    if (o->fri_folding != 2 && o->fri_folding != 4 && o->fri_folding != 8 && o->fri_folding != 16) return -1;
    if (o->fri_rem_max_deg > 255 || !is_pow2((uint64_t)o->fri_rem_max_deg + 1)) return -1;
    if ((uint64_t)o->num_queries >= n * o->blowup) return -1;
    return 0;
}
/* Context::to_elements (RECALLED): TraceInfo [width<<8 | num_aux, n], modulus bytes split in two
 * elements, options [ext<<16 | fold<<8 | rem, grinding, blowup, queries] */
static size_t context_elements(uint64_t n, const orc_options* o, uint64_t* e) {
    e[0] = (uint64_t)W << 8;
    e[1] = n;
    e[2] = 1;           /* LE bytes 01 00 00 00 */
    e[3] = 0xFFFFFFFFULL; /* LE bytes ff ff ff ff */
    e[4] = ((uint64_t)o->field_extension << 16) | ((uint64_t)o->fri_folding << 8) | o->fri_rem_max_deg;
    e[5] = o->grinding;
    e[6] = o->blowup;
    e[7] = o->num_queries;
    return 8;
}
static void write_context(bbuf* w, uint64_t n, const orc_options* o) {
    bb_u8(w, W);            /* main segment width */
    bb_u8(w, 0);            /* aux segments */
    bb_u8(w, (uint8_t)ilog2u(n));
    bb_u16(w, 0);           /* trace meta */
    bb_u8(w, 8);
    bb_u64(w, ORC_P);       /* field modulus LE bytes */
    bb_u8(w, (uint8_t)o->num_queries);
    bb_u8(w, (uint8_t)o->blowup);
    bb_u8(w, (uint8_t)o->grinding);
    bb_u8(w, (uint8_t)o->field_extension);
    bb_u8(w, (uint8_t)o->fri_folding);
    bb_u8(w, (uint8_t)o->fri_rem_max_deg);
}
static uint32_t num_fri_layers(uint64_t N, const orc_options* o) {
    uint64_t maxrem = ((uint64_t)o->fri_rem_max_deg + 1) * o->blowup;
    uint32_t k = 0;
    while (N > maxrem) { N /= o->fri_folding; k++; }
    return k;
}
size_t orc_proof_size_bound(uint64_t n, const orc_options* o) {
    uint64_t N = n * o->blowup, q = o->num_queries, depth = ilog2u(N);
    uint32_t L = num_fri_layers(N, o);
    size_t s = 4096 + q * (W * 8 + 8 + (size_t)L * o->fri_folding * 8);
    s += (size_t)(2 + L) * (1 + q * (1 + depth * 32));
    s += (size_t)(N >> (3 * L)) * 8 + 32 * (L + 3);
    return s;
}

/* FRI fold of one row (apply_drp, RECALLED): values v_k at x*zeta^k (zeta = w_f), interpolate the
 * degree < f polynomial and evaluate it at alpha. x is 7 * w_D^i (constant offset 7 every layer). */
static uint64_t fri_fold_row(const uint64_t* v, uint32_t f, uint64_t x, uint64_t alpha) {
    uint64_t zinv = orc_inv(orc_root(ilog2u(f))), finv = orc_inv(f), c[16];
    for (uint32_t j = 0; j < f; j++) {
        uint64_t s = 0, wj = orc_pow(zinv, j), w = 1;
        for (uint32_t k = 0; k < f; k++) { s = orc_add(s, orc_mul(v[k], w)); w = orc_mul(w, wj); }
        c[j] = orc_mul(s, finv);
    }
    return horner(c, f, orc_mul(alpha, orc_inv(x)));
}
static void fold_positions(const uint64_t* in, uint64_t k, uint64_t target, uint64_t* out, uint64_t* kout) {
    uint64_t m = 0;
    for (uint64_t i = 0; i < k; i++) {
        uint64_t p = in[i] % target;
        int dup = 0;
        for (uint64_t j = 0; j < m; j++) if (out[j] == p) { dup = 1; break; }
        if (!dup) out[m++] = p;
    }
    *kout = m;
}

/* ============================================================ prover */
static int orc_prove_quad(const orc_air* air, const uint64_t* trace, uint64_t n, const orc_options* opt, int faithful,
                          uint8_t* out, size_t* out_len, orc_debug* dbg);
static int orc_verify_quad(const orc_air* air, const uint8_t* proof, size_t len, const orc_options* opt);
int orc_prove(const orc_air* air, const uint64_t* trace, uint64_t n, const orc_options* opt, int faithful,
              uint8_t* out, size_t* out_len, orc_debug* dbg) {
    if (check_options(n, opt)) return ORC_PROVER_ERROR;
    if (opt->field_extension == 2) return orc_prove_quad(air, trace, n, opt, faithful, out, out_len, dbg);
    const uint64_t beta = opt->blowup, N = n * beta, nce = CE_BLOWUP * n, f = opt->fri_folding;
    const uint64_t g = orc_root(ilog2u(n));
    int status = ORC_OK;
    if (t_stage) t_mark = now_ms();

    /* Fiat-Shamir seed: Context::to_elements || pub_inputs.to_elements (ProverChannel::new) */
    uint64_t seed_e[20];
    size_t ne = context_elements(n, opt, seed_e);
    memcpy(seed_e + ne, air->pub, 12 * sizeof(uint64_t));
    coin_t coin;
    coin_init(&coin, seed_e, ne + 12);
    bbuf commitments = {0};

    /* 1. trace: interpolate columns, LDE over 7*<w_N>, row hashes, Merkle (DefaultTraceLde) */
    uint64_t* coef = (uint64_t*)malloc(W * n * sizeof(uint64_t));
    uint64_t* lde = (uint64_t*)malloc(W * N * sizeof(uint64_t)); /* column-major, natural order */
    for (int c = 0; c < W; c++) {
        memcpy(coef + c * n, trace + c * n, n * sizeof(uint64_t));
        orc_interpolate(coef + c * n, n, 1);
        orc_evaluate_lde(coef + c * n, n, beta, ORC_GEN, lde + c * N);
    }
    STAGE(0);
    dg* leaves = (dg*)malloc(N * sizeof(dg));
    for (uint64_t k = 0; k < N; k++) {
        uint64_t row[W];
        for (int c = 0; c < W; c++) row[c] = lde[c * N + k];
        hash_elems(row, W, leaves[k]);
    }
    mtree ttree;
    mtree_build(&ttree, leaves, N);
    bb_put(&commitments, ttree.nodes[1], 32);
    coin_reseed(&coin, ttree.nodes[1]);
    if (dbg) memcpy(dbg->trace_root, ttree.nodes[1], 32);
    STAGE(1);

    /* 2. constraint composition coefficients: 7 transition + 8 boundary */
    uint64_t alpha[W], bcoef[NUM_ASSERT];
    for (int i = 0; i < W; i++) if (coin_draw(&coin, &alpha[i])) status = ORC_PROVER_ERROR;
    for (int i = 0; i < NUM_ASSERT; i++) if (coin_draw(&coin, &bcoef[i])) status = ORC_PROVER_ERROR;

    /* 3. evaluate constraints on the CE domain 7*<w_2n> (DefaultConstraintEvaluator) */
    uint64_t acol[NUM_ASSERT], astep[NUM_ASSERT], aval[NUM_ASSERT];
    air_assertions(air, n, acol, astep, aval);
    uint64_t* ce = (uint64_t*)malloc(nce * sizeof(uint64_t));
    const uint64_t wce = orc_root(ilog2u(nce)), g_last = orc_pow(g, n - 1);
    uint64_t x = ORC_GEN;
    for (uint64_t i = 0; i < nce; i++, x = orc_mul(x, wce)) {
        uint64_t k = i * (beta / CE_BLOWUP), kn = (k + beta) % N, cur[W], nxt[W], r[W];
        for (int c = 0; c < W; c++) { cur[c] = lde[c * N + k]; nxt[c] = lde[c * N + kn]; }
        air_transition(air, cur, nxt, faithful, r);
        uint64_t t = 0;
        for (int c = 0; c < W; c++) t = orc_add(t, orc_mul(alpha[c], r[c]));
        /* transition divisor (x^n - 1)/(x - g^(n-1)) */
        uint64_t zt = orc_mul(orc_sub(orc_pow(x, n), 1), orc_inv(orc_sub(x, g_last)));
        uint64_t acc = orc_mul(t, orc_inv(zt));
        /* boundary groups by step: (x - g^step) */
        uint64_t b0 = 0, b1 = 0;
        for (int a = 0; a < NUM_ASSERT; a++) {
            uint64_t term = orc_mul(bcoef[a], orc_sub(cur[acol[a]], aval[a]));
            if (astep[a] == 0) b0 = orc_add(b0, term); else b1 = orc_add(b1, term);
        }
        acc = orc_add(acc, orc_mul(b0, orc_inv(orc_sub(x, 1))));
        acc = orc_add(acc, orc_mul(b1, orc_inv(orc_sub(x, g_last))));
        ce[i] = acc;
    }
    STAGE(2);

    /* 4. composition polynomial: interpolate over the CE coset, keep num_cols*n = n coefficients
     * (num_constraint_composition_columns = 1 for degree-1 declarations -- RECALLED), LDE, commit */
    orc_interpolate(ce, nce, ORC_GEN);
    uint64_t* hcoef = (uint64_t*)malloc(n * sizeof(uint64_t));
    memcpy(hcoef, ce, n * sizeof(uint64_t));
    uint64_t* hlde = (uint64_t*)malloc(N * sizeof(uint64_t));
    orc_evaluate_lde(hcoef, n, beta, ORC_GEN, hlde);
    for (uint64_t k = 0; k < N; k++) hash_elems(&hlde[k], 1, leaves[k]);
    mtree htree;
    mtree_build(&htree, leaves, N);
    bb_put(&commitments, htree.nodes[1], 32);
    coin_reseed(&coin, htree.nodes[1]);
    if (dbg) memcpy(dbg->constraint_root, htree.nodes[1], 32);
    STAGE(3);

    /* 5. OOD point, frame, DEEP coefficients */
    uint64_t z;
    if (coin_draw(&coin, &z)) status = ORC_PROVER_ERROR;
    uint64_t zg = orc_mul(z, g), ood[2 * W], hz;
    for (int c = 0; c < W; c++) {
        ood[2 * c] = horner(coef + c * n, n, z);
        ood[2 * c + 1] = horner(coef + c * n, n, zg);
    }
    hz = horner(hcoef, n, z);
    uint8_t dtmp[32];
    hash_elems(ood, 2 * W, dtmp);
    coin_reseed(&coin, dtmp);
    hash_elems(&hz, 1, dtmp);
    coin_reseed(&coin, dtmp);
    uint64_t dc[W], gam;
    for (int c = 0; c < W; c++) if (coin_draw(&coin, &dc[c])) status = ORC_PROVER_ERROR;
    if (coin_draw(&coin, &gam)) status = ORC_PROVER_ERROR;
    if (dbg) {
        dbg->z = z;
        for (int c = 0; c < 2 * W; c++) dbg->ood[c] = ood[c];
        dbg->ood[14] = hz;
    }

    /* 6. DEEP composition polynomial in coefficient form (DeepCompositionPoly) */
    uint64_t* t1 = (uint64_t*)calloc(n, sizeof(uint64_t));
    uint64_t* t2 = (uint64_t*)calloc(n, sizeof(uint64_t));
    for (int c = 0; c < W; c++) {
        for (uint64_t j = 0; j < n; j++) {
            uint64_t v = orc_mul(dc[c], coef[c * n + j]);
            t1[j] = orc_add(t1[j], v);
            t2[j] = orc_add(t2[j], v);
        }
        t1[0] = orc_sub(t1[0], orc_mul(dc[c], ood[2 * c]));
        t2[0] = orc_sub(t2[0], orc_mul(dc[c], ood[2 * c + 1]));
    }
    syn_div(t1, n, z);
    syn_div(t2, n, zg);
    for (uint64_t j = 0; j < n; j++) t1[j] = orc_add(t1[j], t2[j]);
    hcoef[0] = orc_sub(hcoef[0], hz);
    syn_div(hcoef, n, z);
    for (uint64_t j = 0; j < n; j++) t1[j] = orc_add(t1[j], orc_mul(gam, hcoef[j]));
    uint64_t deg = 0;
    for (uint64_t j = 0; j < n; j++) if (t1[j]) deg = j;
    if (deg != n - 2) status = ORC_PROVER_ERROR; /* assert_eq!(trace_length - 2, degree) */
    STAGE(4);

    /* 7. FRI layers (FriProver::build_layers) */
    uint32_t nl = num_fri_layers(N, opt);
    uint64_t** layer = (uint64_t**)malloc((nl + 1) * sizeof(uint64_t*));
    mtree* ftree = (mtree*)malloc((nl ? nl : 1) * sizeof(mtree));
    layer[0] = (uint64_t*)malloc(N * sizeof(uint64_t));
    orc_evaluate_lde(t1, n, beta, ORC_GEN, layer[0]);
    uint64_t D = N;
    for (uint32_t l = 0; l < nl; l++) {
        uint64_t rows = D / f;
        for (uint64_t i = 0; i < rows; i++) {
            uint64_t v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = layer[l][i + k * rows];
            hash_elems(v, f, leaves[i]);
        }
        mtree_build(&ftree[l], leaves, rows);
        bb_put(&commitments, ftree[l].nodes[1], 32);
        coin_reseed(&coin, ftree[l].nodes[1]);
        if (dbg) memcpy(dbg->fri_roots[l], ftree[l].nodes[1], 32);
        uint64_t a;
        if (coin_draw(&coin, &a)) status = ORC_PROVER_ERROR;
        layer[l + 1] = (uint64_t*)malloc(rows * sizeof(uint64_t));
        const uint64_t wD = orc_root(ilog2u(D));
        uint64_t xi = ORC_GEN;
        for (uint64_t i = 0; i < rows; i++, xi = orc_mul(xi, wD)) {
            uint64_t v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = layer[l][i + k * rows];
            layer[l + 1][i] = fri_fold_row(v, (uint32_t)f, xi, a);
        }
        D = rows;
    }
    /* remainder: interpolate over 7*<w_D>, keep D/blowup coefficients, commit hash */
    uint64_t* rem = (uint64_t*)malloc(D * sizeof(uint64_t));
    memcpy(rem, layer[nl], D * sizeof(uint64_t));
    orc_interpolate(rem, D, ORC_GEN);
    uint64_t rem_len = D / beta;
    hash_elems(rem, rem_len, dtmp);
    bb_put(&commitments, dtmp, 32);
    coin_reseed(&coin, dtmp);
    if (dbg) { memcpy(dbg->fri_roots[nl], dtmp, 32); dbg->num_fri_layers = nl; }
    STAGE(5);

    /* 8. grinding + query positions (ProverChannel::grind_query_seed / get_query_positions) */
    uint64_t nonce = 1;
    for (;; nonce++) {
        uint8_t h[32];
        merge_int(coin.seed, nonce, h);
        if (tz64(get_le64(h)) >= opt->grinding) break;
    }
    coin_reseed_int(&coin, nonce);
    uint64_t q = opt->num_queries, pos[256];
    for (uint64_t i = 0; i < q; i++) {
        uint8_t h[32];
        coin_next(&coin, h);
        pos[i] = get_le64(h) & (N - 1);
    }
    qsort(pos, q, sizeof(uint64_t), cmp_u64);
    uint64_t nu = 0;
    for (uint64_t i = 0; i < q; i++) if (nu == 0 || pos[nu - 1] != pos[i]) pos[nu++] = pos[i];
    if (dbg) {
        dbg->pow_nonce = nonce;
        dbg->num_unique_queries = (uint32_t)nu;
        for (uint64_t i = 0; i < nu; i++) dbg->positions[i] = pos[i];
    }
    STAGE(6);

    /* 9. proof object + StarkProof::to_bytes (RECALLED layout, DESIGN.md §Proof format) */
    bbuf w = {0}, tmp = {0};
    write_context(&w, n, opt);
    bb_u8(&w, (uint8_t)nu);
    bb_u16(&w, (uint16_t)commitments.n);
    bb_put(&w, commitments.b, commitments.n);
    /* trace queries */
    bb_u8(&w, 1);
    bb_u32(&w, (uint32_t)(nu * W * 8));
    for (uint64_t i = 0; i < nu; i++) for (int c = 0; c < W; c++) bb_u64(&w, lde[c * N + pos[i]]);
    tmp.n = 0;
    mtree_prove_serialize(&ttree, pos, nu, &tmp);
    bb_u32(&w, (uint32_t)tmp.n);
    bb_put(&w, tmp.b, tmp.n);
    /* constraint queries */
    bb_u32(&w, (uint32_t)(nu * 8));
    for (uint64_t i = 0; i < nu; i++) bb_u64(&w, hlde[pos[i]]);
    tmp.n = 0;
    mtree_prove_serialize(&htree, pos, nu, &tmp);
    bb_u32(&w, (uint32_t)tmp.n);
    bb_put(&w, tmp.b, tmp.n);
    /* OOD frame: trace states (frame size byte + interleaved z / z*g values), evaluations */
    bb_u16(&w, (uint16_t)(1 + 2 * W * 8));
    bb_u8(&w, 2);
    for (int c = 0; c < 2 * W; c++) bb_u64(&w, ood[c]);
    bb_u16(&w, 8);
    bb_u64(&w, hz);
    /* FRI proof */
    bb_u8(&w, (uint8_t)nl);
    uint64_t fpos[256], fk = nu;
    memcpy(fpos, pos, nu * sizeof(uint64_t));
    D = N;
    for (uint32_t l = 0; l < nl; l++) {
        uint64_t rows = D / f, np[256], nk;
        fold_positions(fpos, fk, rows, np, &nk);
        bb_u32(&w, (uint32_t)(nk * f * 8));
        for (uint64_t i = 0; i < nk; i++) for (uint64_t k = 0; k < f; k++) bb_u64(&w, layer[l][np[i] + k * rows]);
        tmp.n = 0;
        mtree_prove_serialize(&ftree[l], np, nk, &tmp);
        bb_u32(&w, (uint32_t)tmp.n);
        bb_put(&w, tmp.b, tmp.n);
        memcpy(fpos, np, nk * sizeof(uint64_t));
        fk = nk;
        D = rows;
    }
    bb_u16(&w, (uint16_t)(rem_len * 8));
    for (uint64_t i = 0; i < rem_len; i++) bb_u64(&w, rem[i]);
    bb_u8(&w, 0); /* num_partitions = 1 stored as log2 */
    bb_u64(&w, nonce);

    if (status == ORC_OK) {
        if (!out) *out_len = w.n;
        else if (*out_len < w.n) { *out_len = w.n; status = ORC_BUFFER_TOO_SMALL; }
        else { memcpy(out, w.b, w.n); *out_len = w.n; }
    }
    STAGE(7);
    free(w.b); free(tmp.b); free(commitments.b);
    for (uint32_t l = 0; l <= nl; l++) free(layer[l]);
    for (uint32_t l = 0; l < nl; l++) mtree_free(&ftree[l]);
    free(layer); free(ftree); free(rem);
    free(t1); free(t2); free(hcoef); free(hlde); free(ce); free(leaves); free(coef); free(lde);
    mtree_free(&ttree); mtree_free(&htree);
    return status;
}

/* CPU baseline driver (bench.py cpu_baseline): `count` independent proofs over `threads` OpenMP
 * threads (0 = the OpenMP default), one proof per thread at a time -- the serial batch loop of the
 * reference callers (src/benchmarks/mod.rs:301-342) spread over host cores. Proof bytes are
 * discarded; lens / statuses per proof; stage_ms[ORC_NSTAGE] receives the CPU milliseconds per
 * prover stage summed over all proofs (base-field proofs). Returns the threads that ran. */
int orc_prove_batch(const orc_air* airs, uint32_t count, uint64_t n, const orc_options* opt, int faithful,
                    int threads, size_t* lens, int* statuses, double* stage_ms) {
    int used = 1;
    for (int k = 0; k < ORC_NSTAGE; k++) stage_ms[k] = 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
    {
        double mine[ORC_NSTAGE] = {0};
        t_stage = mine;
        const size_t cap = orc_proof_size_bound(n, opt);
        uint8_t* buf = (uint8_t*)malloc(cap);
        uint64_t* trace = (uint64_t*)malloc(7 * n * sizeof(uint64_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t i = 0; i < (int64_t)count; i++) {
            orc_build_trace(&airs[i], n, trace);
            size_t len = cap;
            statuses[i] = orc_prove(&airs[i], trace, n, opt, faithful, buf, &len, NULL);
            lens[i] = len;
        }
        free(trace);
        free(buf);
        t_stage = NULL;
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            for (int k = 0; k < ORC_NSTAGE; k++) stage_ms[k] += mine[k];
#ifdef _OPENMP
            used = omp_get_num_threads();
#endif
        }
    }
    return used;
}

/* ============================================================ verifier (self-check) */
typedef struct { const uint8_t* p; size_t n, off; int err; } brd;
static const uint8_t* rd(brd* r, size_t k) {
    if (r->err || r->off + k > r->n) { r->err = 1; return NULL; }
    const uint8_t* q = r->p + r->off; r->off += k; return q;
}
static uint64_t rd_u(brd* r, int bytes) {
    const uint8_t* q = rd(r, (size_t)bytes);
    uint64_t v = 0;
    if (q) for (int i = 0; i < bytes; i++) v |= (uint64_t)q[i] << (8 * i);
    return v;
}
/* BatchMerkleProof::get_root restated; leaves given in request order */
static int batch_root(const uint8_t* paths, size_t plen, const uint64_t* idx, uint64_t k, dg* leaf_d, uint64_t depth,
                      uint8_t root[32]) {
    brd r = {paths, plen, 0, 0};
    uint64_t m = rd_u(&r, 1);
    dg** nv = (dg**)calloc(m ? m : 1, sizeof(dg*));
    uint64_t* nvc = (uint64_t*)calloc(m ? m : 1, sizeof(uint64_t));
    for (uint64_t i = 0; i < m; i++) {
        nvc[i] = rd_u(&r, 1);
        nv[i] = (dg*)rd(&r, nvc[i] * 32);
    }
    int bad = r.err || r.off != plen;
    uint64_t* norm = (uint64_t*)malloc((k + 1) * sizeof(uint64_t));
    uint64_t nm = 0;
    for (uint64_t i = 0; i < k; i++) norm[nm++] = idx[i] & ~1ULL;
    qsort(norm, nm, sizeof(uint64_t), cmp_u64);
    uint64_t u = 0;
    for (uint64_t i = 0; i < nm; i++) if (u == 0 || norm[u - 1] != norm[i]) norm[u++] = norm[i];
    nm = u;
    if (nm != m) bad = 1;
    uint64_t* mi = (uint64_t*)malloc((depth + 1) * (nm + 1) * sizeof(uint64_t));
    dg* md = (dg*)malloc((depth + 1) * (nm + 1) * sizeof(dg));
    uint64_t mc = 0;
    uint64_t* cur = (uint64_t*)malloc((nm + 1) * sizeof(uint64_t));
    uint64_t* nxt = (uint64_t*)malloc((nm + 1) * sizeof(uint64_t));
    uint64_t* ptr = (uint64_t*)calloc(nm + 1, sizeof(uint64_t));
    uint64_t L = 1ULL << depth;
    for (uint64_t i = 0; i < nm && !bad; i++) {
        int64_t i1 = -1, i2 = -1;
        for (uint64_t q = 0; q < k; q++) { if (idx[q] == norm[i]) i1 = (int64_t)q; if (idx[q] == norm[i] + 1) i2 = (int64_t)q; }
        uint8_t a[32], b[32];
        if (i1 >= 0) {
            memcpy(a, leaf_d[i1], 32);
            if (i2 >= 0) { memcpy(b, leaf_d[i2], 32); ptr[i] = 0; }
            else { if (nvc[i] < 1) { bad = 1; break; } memcpy(b, nv[i][0], 32); ptr[i] = 1; }
        } else {
            if (nvc[i] < 1 || i2 < 0) { bad = 1; break; }
            memcpy(a, nv[i][0], 32); memcpy(b, leaf_d[i2], 32); ptr[i] = 1;
        }
        mi[mc] = (L + norm[i]) >> 1;
        merge2(a, b, md[mc]);
        cur[i] = mi[mc];
        mc++;
    }
    uint64_t cn = nm;
    for (uint64_t lvl = 1; lvl < depth && !bad; lvl++) {
        uint64_t nn = 0;
        for (uint64_t i = 0; i < cn && !bad; i++) {
            uint64_t node = cur[i], sib = node ^ 1;
            uint8_t sd[32], nd[32];
            int found = 0;
            if (i + 1 < cn && cur[i + 1] == sib) {
                i++;
                for (uint64_t s = mc; s-- > 0;) if (mi[s] == sib) { memcpy(sd, md[s], 32); found = 1; break; }
                if (!found) { bad = 1; break; }
            } else {
                if (ptr[i] >= nvc[i]) { bad = 1; break; }
                memcpy(sd, nv[i][ptr[i]++], 32);
            }
            found = 0;
            for (uint64_t s = mc; s-- > 0;) if (mi[s] == node) { memcpy(nd, md[s], 32); found = 1; break; }
            if (!found) { bad = 1; break; }
            mi[mc] = node >> 1;
            if (node & 1) merge2(sd, nd, md[mc]); else merge2(nd, sd, md[mc]);
            nxt[nn++] = mi[mc];
            mc++;
        }
        uint64_t* t = cur; cur = nxt; nxt = t; cn = nn;
    }
    if (!bad) {
        int found = 0;
        for (uint64_t s = mc; s-- > 0;) if (mi[s] == 1) { memcpy(root, md[s], 32); found = 1; break; }
        if (!found) bad = 1;
    }
    free(nv); free(nvc); free(norm); free(mi); free(md); free(cur); free(nxt); free(ptr);
    return bad ? -1 : 0;
}

int orc_verify(const orc_air* air, const uint8_t* proof, size_t len, const orc_options* opt) {
    if (opt->field_extension == 2) return orc_verify_quad(air, proof, len, opt);
    brd r = {proof, len, 0, 0};
    /* context */
    uint64_t width = rd_u(&r, 1), naux = rd_u(&r, 1), logn = rd_u(&r, 1), meta = rd_u(&r, 2);
    rd(&r, meta);
    uint64_t mlen = rd_u(&r, 1), modulus = rd_u(&r, 8);
    orc_options o;
    o.num_queries = (uint32_t)rd_u(&r, 1); o.blowup = (uint32_t)rd_u(&r, 1); o.grinding = (uint32_t)rd_u(&r, 1);
    o.field_extension = (uint32_t)rd_u(&r, 1); o.fri_folding = (uint32_t)rd_u(&r, 1); o.fri_rem_max_deg = (uint32_t)rd_u(&r, 1);
    if (r.err || width != W || naux != 0 || mlen != 8 || modulus != ORC_P || logn > 26) return ORC_VERIFY_FAILED;
    if (memcmp(&o, opt, sizeof o)) return ORC_VERIFY_FAILED; /* AcceptableOptions::OptionSet([options]) */
    uint64_t n = 1ULL << logn;
    if (check_options(n, &o)) return ORC_VERIFY_FAILED;
    const uint64_t beta = o.blowup, N = n * beta, f = o.fri_folding, depth = ilog2u(N);
    const uint64_t g = orc_root((unsigned)logn);
    uint32_t nl = num_fri_layers(N, &o);
    uint64_t nu = rd_u(&r, 1);
    uint64_t clen = rd_u(&r, 2);
    const uint8_t* com = rd(&r, clen);
    if (r.err || clen != 32ULL * (3 + nl) || nu == 0) return ORC_VERIFY_FAILED;
    if (rd_u(&r, 1) != 1) return ORC_VERIFY_FAILED;
    uint64_t tvl = rd_u(&r, 4); const uint8_t* tv = rd(&r, tvl);
    uint64_t tpl = rd_u(&r, 4); const uint8_t* tp = rd(&r, tpl);
    uint64_t cvl = rd_u(&r, 4); const uint8_t* cv = rd(&r, cvl);
    uint64_t cpl = rd_u(&r, 4); const uint8_t* cp = rd(&r, cpl);
    uint64_t osl = rd_u(&r, 2); const uint8_t* os = rd(&r, osl);
    uint64_t oel = rd_u(&r, 2); const uint8_t* oe = rd(&r, oel);
    if (r.err || tvl != nu * W * 8 || cvl != nu * 8 || osl != 1 + 2 * W * 8 || oel != 8 || os[0] != 2)
        return ORC_VERIFY_FAILED;
    uint64_t nfl = rd_u(&r, 1);
    if (nfl != nl) return ORC_VERIFY_FAILED;
    const uint8_t *fv[16], *fp[16];
    uint64_t fvl[16], fpl[16];
    for (uint32_t l = 0; l < nl; l++) {
        fvl[l] = rd_u(&r, 4); fv[l] = rd(&r, fvl[l]);
        fpl[l] = rd_u(&r, 4); fp[l] = rd(&r, fpl[l]);
    }
    uint64_t rml = rd_u(&r, 2); const uint8_t* rm = rd(&r, rml);
    uint64_t parts = rd_u(&r, 1);
    uint64_t nonce = rd_u(&r, 8);
    if (r.err || r.off != len || parts != 0) return ORC_VERIFY_FAILED;

    /* transcript */
    uint64_t seed_e[20];
    size_t ne = context_elements(n, &o, seed_e);
    memcpy(seed_e + ne, air->pub, 12 * sizeof(uint64_t));
    coin_t coin;
    coin_init(&coin, seed_e, ne + 12);
    coin_reseed(&coin, com);
    uint64_t alpha[W], bcoef[NUM_ASSERT], z, dc[W], gam;
    for (int i = 0; i < W; i++) if (coin_draw(&coin, &alpha[i])) return ORC_VERIFY_FAILED;
    for (int i = 0; i < NUM_ASSERT; i++) if (coin_draw(&coin, &bcoef[i])) return ORC_VERIFY_FAILED;
    coin_reseed(&coin, com + 32);
    if (coin_draw(&coin, &z)) return ORC_VERIFY_FAILED;
    uint64_t ood[2 * W], hz = get_le64(oe), zg = orc_mul(z, g);
    for (int c = 0; c < 2 * W; c++) ood[c] = get_le64(os + 1 + 8 * c);
    /* OOD consistency: constraint composition at z from the frame (evaluate_constraints) */
    {
        uint64_t cur[W], nxt[W], rr[W], acol[NUM_ASSERT], astep[NUM_ASSERT], aval[NUM_ASSERT];
        for (int c = 0; c < W; c++) { cur[c] = ood[2 * c]; nxt[c] = ood[2 * c + 1]; }
        air_transition(air, cur, nxt, 0, rr);
        uint64_t t = 0;
        for (int c = 0; c < W; c++) t = orc_add(t, orc_mul(alpha[c], rr[c]));
        uint64_t g_last = orc_pow(g, n - 1);
        uint64_t e = orc_mul(orc_mul(t, orc_sub(z, g_last)), orc_inv(orc_sub(orc_pow(z, n), 1)));
        air_assertions(air, n, acol, astep, aval);
        uint64_t b0 = 0, b1 = 0;
        for (int a = 0; a < NUM_ASSERT; a++) {
            uint64_t term = orc_mul(bcoef[a], orc_sub(cur[acol[a]], aval[a]));
            if (astep[a] == 0) b0 = orc_add(b0, term); else b1 = orc_add(b1, term);
        }
        e = orc_add(e, orc_mul(b0, orc_inv(orc_sub(z, 1))));
        e = orc_add(e, orc_mul(b1, orc_inv(orc_sub(z, g_last))));
        if (e != hz) return ORC_VERIFY_FAILED;
    }
    uint8_t dtmp[32];
    hash_elems(ood, 2 * W, dtmp);
    coin_reseed(&coin, dtmp);
    hash_elems(&hz, 1, dtmp);
    coin_reseed(&coin, dtmp);
    for (int c = 0; c < W; c++) if (coin_draw(&coin, &dc[c])) return ORC_VERIFY_FAILED;
    if (coin_draw(&coin, &gam)) return ORC_VERIFY_FAILED;
    uint64_t falpha[16];
    for (uint32_t l = 0; l <= nl; l++) {
        coin_reseed(&coin, com + 64 + 32 * l);
        uint64_t a;
        if (coin_draw(&coin, &a)) return ORC_VERIFY_FAILED;
        if (l < nl) falpha[l] = a;
    }
    {
        uint8_t h[32];
        merge_int(coin.seed, nonce, h);
        if (tz64(get_le64(h)) < o.grinding) return ORC_VERIFY_FAILED;
    }
    coin_reseed_int(&coin, nonce);
    uint64_t pos[256], q = o.num_queries;
    for (uint64_t i = 0; i < q; i++) { uint8_t h[32]; coin_next(&coin, h); pos[i] = get_le64(h) & (N - 1); }
    qsort(pos, q, sizeof(uint64_t), cmp_u64);
    uint64_t u = 0;
    for (uint64_t i = 0; i < q; i++) if (u == 0 || pos[u - 1] != pos[i]) pos[u++] = pos[i];
    if (u != nu) return ORC_VERIFY_FAILED;

    int ok = 1;
    dg* ld = (dg*)malloc(256 * sizeof(dg));
    uint8_t root[32];
    /* trace + constraint openings */
    for (uint64_t i = 0; i < nu; i++) orc_blake3(tv + i * W * 8, W * 8, ld[i]);
    if (batch_root(tp, tpl, pos, nu, ld, depth, root) || memcmp(root, com, 32)) ok = 0;
    for (uint64_t i = 0; i < nu; i++) orc_blake3(cv + i * 8, 8, ld[i]);
    if (ok && (batch_root(cp, cpl, pos, nu, ld, depth, root) || memcmp(root, com + 32, 32))) ok = 0;
    /* DEEP evaluations at the query points */
    uint64_t ev[256];
    const uint64_t wN = orc_root((unsigned)depth);
    for (uint64_t i = 0; i < nu && ok; i++) {
        uint64_t x = orc_mul(ORC_GEN, orc_pow(wN, pos[i]));
        uint64_t s1 = 0, s2 = 0;
        for (int c = 0; c < W; c++) {
            uint64_t tx = get_le64(tv + (i * W + c) * 8);
            s1 = orc_add(s1, orc_mul(dc[c], orc_sub(tx, ood[2 * c])));
            s2 = orc_add(s2, orc_mul(dc[c], orc_sub(tx, ood[2 * c + 1])));
        }
        uint64_t hx = get_le64(cv + i * 8);
        uint64_t izx = orc_inv(orc_sub(x, z));
        ev[i] = orc_add(orc_mul(s1, izx), orc_mul(s2, orc_inv(orc_sub(x, zg))));
        ev[i] = orc_add(ev[i], orc_mul(orc_mul(gam, orc_sub(hx, hz)), izx));
    }
    /* FRI */
    uint64_t D = N, cp_pos[256], ck = nu;
    memcpy(cp_pos, pos, nu * sizeof(uint64_t));
    for (uint32_t l = 0; l < nl && ok; l++) {
        uint64_t rows = D / f, np[256], nk;
        fold_positions(cp_pos, ck, rows, np, &nk);
        if (fvl[l] != nk * f * 8) { ok = 0; break; }
        for (uint64_t i = 0; i < nk; i++) orc_blake3(fv[l] + i * f * 8, f * 8, ld[i]);
        if (batch_root(fp[l], fpl[l], np, nk, ld, ilog2u(rows), root) || memcmp(root, com + 64 + 32 * l, 32)) { ok = 0; break; }
        for (uint64_t i = 0; i < ck; i++) {
            uint64_t ri = cp_pos[i] % rows, e = cp_pos[i] / rows, idx = 0;
            while (np[idx] != ri) idx++;
            if (get_le64(fv[l] + (idx * f + e) * 8) != ev[i]) { ok = 0; break; }
        }
        const uint64_t wD = orc_root(ilog2u(D));
        for (uint64_t i = 0; i < nk && ok; i++) {
            uint64_t v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = get_le64(fv[l] + (i * f + k) * 8);
            ev[i] = fri_fold_row(v, (uint32_t)f, orc_mul(ORC_GEN, orc_pow(wD, np[i])), falpha[l]);
        }
        memcpy(cp_pos, np, nk * sizeof(uint64_t));
        ck = nk;
        D = rows;
    }
    if (ok) {
        uint64_t rl = rml / 8, remc[4096];
        if (rml % 8 || rl == 0 || rl != D / beta || rl > 4096) ok = 0;
        for (uint64_t i = 0; ok && i < rl; i++) remc[i] = get_le64(rm + 8 * i);
        if (ok) { hash_elems(remc, rl, dtmp); if (memcmp(dtmp, com + 64 + 32 * nl, 32)) ok = 0; }
        const uint64_t wD = orc_root(ilog2u(D));
        for (uint64_t i = 0; ok && i < ck; i++)
            if (horner(remc, rl, orc_mul(ORC_GEN, orc_pow(wD, cp_pos[i]))) != ev[i]) ok = 0;
    }
    free(ld);
    return ok ? ORC_OK : ORC_VERIFY_FAILED;
}

/* ============================================================ quadratic extension (RECALLED)
 * FieldExtension::Quadratic of winter-math f64: E = F[phi]/(phi^2 - phi + 2), elements a + b phi
 * serialised as (a, b) canonical LE u64s. With it the trace and its commitment stay in the base
 * field; the composition coefficients, the OOD point z, the DEEP coefficients and the FRI
 * alphas are drawn as E (16 digest bytes -> two elements, retry if either is >= p); constraint
 * evaluations, composition polynomial, OOD frame, DEEP polynomial, FRI layers and remainder are
 * E-valued. Base-field linear maps (NTTs, the iDFT of a FRI fold) act per coordinate. */
typedef struct { uint64_t a, b; } fq;
static fq fq_make(uint64_t a, uint64_t b) { fq r; r.a = a; r.b = b; return r; }
static fq fq_add(fq x, fq y) { return fq_make(orc_add(x.a, y.a), orc_add(x.b, y.b)); }
static fq fq_sub(fq x, fq y) { return fq_make(orc_sub(x.a, y.a), orc_sub(x.b, y.b)); }
static fq fq_mulb(fq x, uint64_t s) { return fq_make(orc_mul(x.a, s), orc_mul(x.b, s)); }
static fq fq_mul(fq x, fq y) {
    /* (a0 + a1 phi)(b0 + b1 phi) = a0 b0 - 2 a1 b1 + (a0 b1 + a1 b0 + a1 b1) phi */
    uint64_t a0b0 = orc_mul(x.a, y.a), a1b1 = orc_mul(x.b, y.b);
    uint64_t cross = orc_add(orc_add(orc_mul(x.a, y.b), orc_mul(x.b, y.a)), a1b1);
    return fq_make(orc_sub(a0b0, orc_add(a1b1, a1b1)), cross);
}
static fq fq_inv(fq x) {
    /* x^-1 = frob(x) / (x frob(x)), frob(a + b phi) = (a + b) - b phi, the norm is in F */
    fq f = fq_make(orc_add(x.a, x.b), orc_sub(0, x.b));
    fq nrm = fq_mul(x, f);
    return fq_mulb(f, orc_inv(nrm.a));
}
static int fq_eq(fq x, fq y) { return x.a == y.a && x.b == y.b; }
static int fq_is_zero(fq x) { return x.a == 0 && x.b == 0; }
static int coin_draw_fq(coin_t* c, fq* out) {
    for (int i = 0; i < 1000; i++) {
        uint8_t h[32];
        coin_next(c, h);
        uint64_t a = get_le64(h), b = get_le64(h + 8);
        if (a < ORC_P && b < ORC_P) { *out = fq_make(a, b); return 0; }
    }
    return -1;
}
static void hash_fq(const fq* e, size_t cnt, uint8_t out[32]) {
    uint8_t* buf = (uint8_t*)malloc(cnt * 16 + 1);
    for (size_t i = 0; i < cnt; i++) { put_le64(buf + 16 * i, e[i].a); put_le64(buf + 16 * i + 8, e[i].b); }
    orc_blake3(buf, cnt * 16, out);
    free(buf);
}
static void bb_fq(bbuf* w, fq v) { bb_u64(w, v.a); bb_u64(w, v.b); }
static fq horner_bq(const uint64_t* c, uint64_t n, fq x) { /* base coefficients at an E point */
    fq r = fq_make(0, 0);
    for (uint64_t j = n; j-- > 0;) r = fq_add(fq_mul(r, x), fq_make(c[j], 0));
    return r;
}
static fq horner_q(const fq* c, uint64_t n, fq x) {
    fq r = fq_make(0, 0);
    for (uint64_t j = n; j-- > 0;) r = fq_add(fq_mul(r, x), c[j]);
    return r;
}
static void syn_div_q(fq* a, uint64_t n, fq b) {
    fq c = fq_make(0, 0);
    for (uint64_t j = n; j-- > 0;) {
        fq v = fq_add(a[j], fq_mul(b, c));
        a[j] = c;
        c = v;
    }
}
/* per-coordinate NTT helpers over fq arrays */
static void split_q(const fq* v, uint64_t n, uint64_t* x, uint64_t* y) {
    for (uint64_t i = 0; i < n; i++) { x[i] = v[i].a; y[i] = v[i].b; }
}
static void join_q(const uint64_t* x, const uint64_t* y, uint64_t n, fq* v) {
    for (uint64_t i = 0; i < n; i++) v[i] = fq_make(x[i], y[i]);
}
static void interpolate_q(fq* v, uint64_t n, uint64_t offset) {
    uint64_t* x = (uint64_t*)malloc(n * 8);
    uint64_t* y = (uint64_t*)malloc(n * 8);
    split_q(v, n, x, y);
    orc_interpolate(x, n, offset);
    orc_interpolate(y, n, offset);
    join_q(x, y, n, v);
    free(x); free(y);
}
static void lde_q(const fq* c, uint64_t n, uint64_t blowup, fq* out) {
    uint64_t N = n * blowup;
    uint64_t* x = (uint64_t*)malloc(n * 8);
    uint64_t* y = (uint64_t*)malloc(n * 8);
    uint64_t* X = (uint64_t*)malloc(N * 8);
    uint64_t* Y = (uint64_t*)malloc(N * 8);
    split_q(c, n, x, y);
    orc_evaluate_lde(x, n, blowup, ORC_GEN, X);
    orc_evaluate_lde(y, n, blowup, ORC_GEN, Y);
    join_q(X, Y, N, out);
    free(x); free(y); free(X); free(Y);
}
static fq fri_fold_row_q(const fq* v, uint32_t f, uint64_t x, fq alpha) {
    uint64_t zinv = orc_inv(orc_root(ilog2u(f))), finv = orc_inv(f);
    fq c[16];
    for (uint32_t j = 0; j < f; j++) {
        fq s = fq_make(0, 0);
        uint64_t wj = orc_pow(zinv, j), w = 1;
        for (uint32_t k = 0; k < f; k++) { s = fq_add(s, fq_mulb(v[k], w)); w = orc_mul(w, wj); }
        c[j] = fq_mulb(s, finv);
    }
    return horner_q(c, f, fq_mulb(alpha, orc_inv(x)));
}
static void air_transition_q(const orc_air* air, const fq cur[7], const fq nxt[7], fq r[7]) {
    uint64_t large = orc_mul(STANDARD_BURN, 1000);
    r[0] = fq_mul(fq_sub(cur[0], fq_make(STANDARD_BURN, 0)), fq_sub(cur[0], fq_make(large, 0)));
    r[1] = fq_sub(cur[1], cur[0]);
    r[2] = fq_sub(cur[2], fq_make((uint32_t)air->pub[PI_TXN], 0));
    r[3] = fq_sub(cur[3], fq_make((uint32_t)air->pub[PI_RH], 0));
    fq d = fq_sub(nxt[4], cur[4]);
    r[4] = fq_mul(d, fq_sub(d, fq_make(1, 0)));
    r[5] = fq_sub(cur[5], fq_make(air->nullifier, 0));
    r[6] = fq_sub(cur[6], fq_make(air->commitment, 0));
}

static int orc_prove_quad(const orc_air* air, const uint64_t* trace, uint64_t n, const orc_options* opt, int faithful,
                          uint8_t* out, size_t* out_len, orc_debug* dbg) {
    const uint64_t beta = opt->blowup, N = n * beta, nce = CE_BLOWUP * n, f = opt->fri_folding;
    const uint64_t g = orc_root(ilog2u(n));
    int status = ORC_OK;
    uint64_t seed_e[20];
    size_t ne = context_elements(n, opt, seed_e);
    memcpy(seed_e + ne, air->pub, 12 * sizeof(uint64_t));
    coin_t coin;
    coin_init(&coin, seed_e, ne + 12);
    bbuf commitments = {0};

    /* 1. trace (base field, as without extension) */
    uint64_t* coef = (uint64_t*)malloc(W * n * sizeof(uint64_t));
    uint64_t* lde = (uint64_t*)malloc(W * N * sizeof(uint64_t));
    for (int c = 0; c < W; c++) {
        memcpy(coef + c * n, trace + c * n, n * sizeof(uint64_t));
        orc_interpolate(coef + c * n, n, 1);
        orc_evaluate_lde(coef + c * n, n, beta, ORC_GEN, lde + c * N);
    }
    dg* leaves = (dg*)malloc(N * sizeof(dg));
    for (uint64_t k = 0; k < N; k++) {
        uint64_t row[W];
        for (int c = 0; c < W; c++) row[c] = lde[c * N + k];
        hash_elems(row, W, leaves[k]);
    }
    mtree ttree;
    mtree_build(&ttree, leaves, N);
    bb_put(&commitments, ttree.nodes[1], 32);
    coin_reseed(&coin, ttree.nodes[1]);

    /* 2. composition coefficients in E */
    fq alpha[W], bcoef[NUM_ASSERT];
    for (int i = 0; i < W; i++) if (coin_draw_fq(&coin, &alpha[i])) status = ORC_PROVER_ERROR;
    for (int i = 0; i < NUM_ASSERT; i++) if (coin_draw_fq(&coin, &bcoef[i])) status = ORC_PROVER_ERROR;

    /* 3. constraint evaluations (E) on the CE coset */
    uint64_t acol[NUM_ASSERT], astep[NUM_ASSERT], aval[NUM_ASSERT];
    air_assertions(air, n, acol, astep, aval);
    fq* ce = (fq*)malloc(nce * sizeof(fq));
    const uint64_t wce = orc_root(ilog2u(nce)), g_last = orc_pow(g, n - 1);
    uint64_t x = ORC_GEN;
    for (uint64_t i = 0; i < nce; i++, x = orc_mul(x, wce)) {
        uint64_t k = i * (beta / CE_BLOWUP), kn = (k + beta) % N, cur[W], nxt[W], r[W];
        for (int c = 0; c < W; c++) { cur[c] = lde[c * N + k]; nxt[c] = lde[c * N + kn]; }
        air_transition(air, cur, nxt, faithful, r);
        fq t = fq_make(0, 0);
        for (int c = 0; c < W; c++) t = fq_add(t, fq_mulb(alpha[c], r[c]));
        uint64_t zt = orc_mul(orc_sub(orc_pow(x, n), 1), orc_inv(orc_sub(x, g_last)));
        fq acc = fq_mulb(t, orc_inv(zt));
        fq b0 = fq_make(0, 0), b1 = fq_make(0, 0);
        for (int a = 0; a < NUM_ASSERT; a++) {
            fq term = fq_mulb(bcoef[a], orc_sub(cur[acol[a]], aval[a]));
            if (astep[a] == 0) b0 = fq_add(b0, term); else b1 = fq_add(b1, term);
        }
        acc = fq_add(acc, fq_mulb(b0, orc_inv(orc_sub(x, 1))));
        acc = fq_add(acc, fq_mulb(b1, orc_inv(orc_sub(x, g_last))));
        ce[i] = acc;
    }

    /* 4. composition polynomial (E), LDE per coordinate, leaves = hash of one E element */
    interpolate_q(ce, nce, ORC_GEN);
    fq* hcoef = (fq*)malloc(n * sizeof(fq));
    memcpy(hcoef, ce, n * sizeof(fq));
    fq* hlde = (fq*)malloc(N * sizeof(fq));
    lde_q(hcoef, n, beta, hlde);
    for (uint64_t k = 0; k < N; k++) hash_fq(&hlde[k], 1, leaves[k]);
    mtree htree;
    mtree_build(&htree, leaves, N);
    bb_put(&commitments, htree.nodes[1], 32);
    coin_reseed(&coin, htree.nodes[1]);

    /* 5. OOD point z in E, frame, DEEP coefficients */
    fq z;
    if (coin_draw_fq(&coin, &z)) status = ORC_PROVER_ERROR;
    fq zg = fq_mulb(z, g), ood[2 * W], hz;
    for (int c = 0; c < W; c++) {
        ood[2 * c] = horner_bq(coef + c * n, n, z);
        ood[2 * c + 1] = horner_bq(coef + c * n, n, zg);
    }
    hz = horner_q(hcoef, n, z);
    uint8_t dtmp[32];
    hash_fq(ood, 2 * W, dtmp);
    coin_reseed(&coin, dtmp);
    hash_fq(&hz, 1, dtmp);
    coin_reseed(&coin, dtmp);
    fq dc[W], gam;
    for (int c = 0; c < W; c++) if (coin_draw_fq(&coin, &dc[c])) status = ORC_PROVER_ERROR;
    if (coin_draw_fq(&coin, &gam)) status = ORC_PROVER_ERROR;
    if (dbg) {
        dbg->z = z.a;
        for (int c = 0; c < 2 * W; c++) dbg->ood[c] = ood[c].a;
        dbg->ood[14] = hz.a;
    }

    /* 6. DEEP composition polynomial (E coefficients) */
    fq* t1 = (fq*)calloc(n, sizeof(fq));
    fq* t2 = (fq*)calloc(n, sizeof(fq));
    for (int c = 0; c < W; c++) {
        for (uint64_t j = 0; j < n; j++) {
            fq v = fq_mulb(dc[c], coef[c * n + j]);
            t1[j] = fq_add(t1[j], v);
            t2[j] = fq_add(t2[j], v);
        }
        t1[0] = fq_sub(t1[0], fq_mul(dc[c], ood[2 * c]));
        t2[0] = fq_sub(t2[0], fq_mul(dc[c], ood[2 * c + 1]));
    }
    syn_div_q(t1, n, z);
    syn_div_q(t2, n, zg);
    for (uint64_t j = 0; j < n; j++) t1[j] = fq_add(t1[j], t2[j]);
    hcoef[0] = fq_sub(hcoef[0], hz);
    syn_div_q(hcoef, n, z);
    for (uint64_t j = 0; j < n; j++) t1[j] = fq_add(t1[j], fq_mul(gam, hcoef[j]));
    uint64_t deg = 0;
    for (uint64_t j = 0; j < n; j++) if (!fq_is_zero(t1[j])) deg = j;
    if (deg != n - 2) status = ORC_PROVER_ERROR;

    /* 7. FRI over E values */
    uint32_t nl = num_fri_layers(N, opt);
    fq** layer = (fq**)malloc((nl + 1) * sizeof(fq*));
    mtree* ftree = (mtree*)malloc((nl ? nl : 1) * sizeof(mtree));
    layer[0] = (fq*)malloc(N * sizeof(fq));
    lde_q(t1, n, beta, layer[0]);
    uint64_t D = N;
    for (uint32_t l = 0; l < nl; l++) {
        uint64_t rows = D / f;
        for (uint64_t i = 0; i < rows; i++) {
            fq v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = layer[l][i + k * rows];
            hash_fq(v, f, leaves[i]);
        }
        mtree_build(&ftree[l], leaves, rows);
        bb_put(&commitments, ftree[l].nodes[1], 32);
        coin_reseed(&coin, ftree[l].nodes[1]);
        fq a;
        if (coin_draw_fq(&coin, &a)) status = ORC_PROVER_ERROR;
        layer[l + 1] = (fq*)malloc(rows * sizeof(fq));
        const uint64_t wD = orc_root(ilog2u(D));
        uint64_t xi = ORC_GEN;
        for (uint64_t i = 0; i < rows; i++, xi = orc_mul(xi, wD)) {
            fq v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = layer[l][i + k * rows];
            layer[l + 1][i] = fri_fold_row_q(v, (uint32_t)f, xi, a);
        }
        D = rows;
    }
    fq* rem = (fq*)malloc(D * sizeof(fq));
    memcpy(rem, layer[nl], D * sizeof(fq));
    interpolate_q(rem, D, ORC_GEN);
    uint64_t rem_len = D / beta;
    hash_fq(rem, rem_len, dtmp);
    bb_put(&commitments, dtmp, 32);
    coin_reseed(&coin, dtmp);

    /* 8. grinding + query positions */
    uint64_t nonce = 1;
    for (;; nonce++) {
        uint8_t h[32];
        merge_int(coin.seed, nonce, h);
        if (tz64(get_le64(h)) >= opt->grinding) break;
    }
    coin_reseed_int(&coin, nonce);
    uint64_t q = opt->num_queries, pos[256];
    for (uint64_t i = 0; i < q; i++) {
        uint8_t h[32];
        coin_next(&coin, h);
        pos[i] = get_le64(h) & (N - 1);
    }
    qsort(pos, q, sizeof(uint64_t), cmp_u64);
    uint64_t nu = 0;
    for (uint64_t i = 0; i < q; i++) if (nu == 0 || pos[nu - 1] != pos[i]) pos[nu++] = pos[i];
    if (dbg) {
        dbg->pow_nonce = nonce;
        dbg->num_unique_queries = (uint32_t)nu;
        for (uint64_t i = 0; i < nu; i++) dbg->positions[i] = pos[i];
        dbg->num_fri_layers = nl;
    }

    /* 9. StarkProof::to_bytes with 16-byte E elements */
    bbuf w = {0}, tmp = {0};
    write_context(&w, n, opt);
    bb_u8(&w, (uint8_t)nu);
    bb_u16(&w, (uint16_t)commitments.n);
    bb_put(&w, commitments.b, commitments.n);
    bb_u8(&w, 1);
    bb_u32(&w, (uint32_t)(nu * W * 8));
    for (uint64_t i = 0; i < nu; i++) for (int c = 0; c < W; c++) bb_u64(&w, lde[c * N + pos[i]]);
    tmp.n = 0;
    mtree_prove_serialize(&ttree, pos, nu, &tmp);
    bb_u32(&w, (uint32_t)tmp.n);
    bb_put(&w, tmp.b, tmp.n);
    bb_u32(&w, (uint32_t)(nu * 16));
    for (uint64_t i = 0; i < nu; i++) bb_fq(&w, hlde[pos[i]]);
    tmp.n = 0;
    mtree_prove_serialize(&htree, pos, nu, &tmp);
    bb_u32(&w, (uint32_t)tmp.n);
    bb_put(&w, tmp.b, tmp.n);
    bb_u16(&w, (uint16_t)(1 + 2 * W * 16));
    bb_u8(&w, 2);
    for (int c = 0; c < 2 * W; c++) bb_fq(&w, ood[c]);
    bb_u16(&w, 16);
    bb_fq(&w, hz);
    bb_u8(&w, (uint8_t)nl);
    uint64_t fpos[256], fk = nu;
    memcpy(fpos, pos, nu * sizeof(uint64_t));
    D = N;
    for (uint32_t l = 0; l < nl; l++) {
        uint64_t rows = D / f, np[256], nk;
        fold_positions(fpos, fk, rows, np, &nk);
        bb_u32(&w, (uint32_t)(nk * f * 16));
        for (uint64_t i = 0; i < nk; i++) for (uint64_t k = 0; k < f; k++) bb_fq(&w, layer[l][np[i] + k * rows]);
        tmp.n = 0;
        mtree_prove_serialize(&ftree[l], np, nk, &tmp);
        bb_u32(&w, (uint32_t)tmp.n);
        bb_put(&w, tmp.b, tmp.n);
        memcpy(fpos, np, nk * sizeof(uint64_t));
        fk = nk;
        D = rows;
    }
    bb_u16(&w, (uint16_t)(rem_len * 16));
    for (uint64_t i = 0; i < rem_len; i++) bb_fq(&w, rem[i]);
    bb_u8(&w, 0);
    bb_u64(&w, nonce);

    if (status == ORC_OK) {
        if (!out) *out_len = w.n;
        else if (*out_len < w.n) { *out_len = w.n; status = ORC_BUFFER_TOO_SMALL; }
        else { memcpy(out, w.b, w.n); *out_len = w.n; }
    }
    free(w.b); free(tmp.b); free(commitments.b);
    for (uint32_t l = 0; l <= nl; l++) free(layer[l]);
    for (uint32_t l = 0; l < nl; l++) mtree_free(&ftree[l]);
    free(layer); free(ftree); free(rem);
    free(t1); free(t2); free(hcoef); free(hlde); free(ce); free(leaves); free(coef); free(lde);
    mtree_free(&ttree); mtree_free(&htree);
    return status;
}

static fq rd_fq(const uint8_t* p) { return fq_make(get_le64(p), get_le64(p + 8)); }
static int orc_verify_quad(const orc_air* air, const uint8_t* proof, size_t len, const orc_options* opt) {
    brd r = {proof, len, 0, 0};
    uint64_t width = rd_u(&r, 1), naux = rd_u(&r, 1), logn = rd_u(&r, 1), meta = rd_u(&r, 2);
    rd(&r, meta);
    uint64_t mlen = rd_u(&r, 1), modulus = rd_u(&r, 8);
    orc_options o;
    o.num_queries = (uint32_t)rd_u(&r, 1); o.blowup = (uint32_t)rd_u(&r, 1); o.grinding = (uint32_t)rd_u(&r, 1);
    o.field_extension = (uint32_t)rd_u(&r, 1); o.fri_folding = (uint32_t)rd_u(&r, 1); o.fri_rem_max_deg = (uint32_t)rd_u(&r, 1);
    if (r.err || width != W || naux != 0 || mlen != 8 || modulus != ORC_P || logn > 26) return ORC_VERIFY_FAILED;
    if (memcmp(&o, opt, sizeof o)) return ORC_VERIFY_FAILED;
    uint64_t n = 1ULL << logn;
    if (check_options(n, &o)) return ORC_VERIFY_FAILED;
    const uint64_t beta = o.blowup, N = n * beta, f = o.fri_folding, depth = ilog2u(N);
    const uint64_t g = orc_root((unsigned)logn);
    uint32_t nl = num_fri_layers(N, &o);
    uint64_t nu = rd_u(&r, 1);
    uint64_t clen = rd_u(&r, 2);
    const uint8_t* com = rd(&r, clen);
    if (r.err || clen != 32ULL * (3 + nl) || nu == 0) return ORC_VERIFY_FAILED;
    if (rd_u(&r, 1) != 1) return ORC_VERIFY_FAILED;
    uint64_t tvl = rd_u(&r, 4); const uint8_t* tv = rd(&r, tvl);
    uint64_t tpl = rd_u(&r, 4); const uint8_t* tp = rd(&r, tpl);
    uint64_t cvl = rd_u(&r, 4); const uint8_t* cv = rd(&r, cvl);
    uint64_t cpl = rd_u(&r, 4); const uint8_t* cp = rd(&r, cpl);
    uint64_t osl = rd_u(&r, 2); const uint8_t* os = rd(&r, osl);
    uint64_t oel = rd_u(&r, 2); const uint8_t* oe = rd(&r, oel);
    if (r.err || tvl != nu * W * 8 || cvl != nu * 16 || osl != 1 + 2 * W * 16 || oel != 16 || os[0] != 2)
        return ORC_VERIFY_FAILED;
    uint64_t nfl = rd_u(&r, 1);
    if (nfl != nl) return ORC_VERIFY_FAILED;
    const uint8_t *fv[16], *fp[16];
    uint64_t fvl[16], fpl[16];
    for (uint32_t l = 0; l < nl; l++) {
        fvl[l] = rd_u(&r, 4); fv[l] = rd(&r, fvl[l]);
        fpl[l] = rd_u(&r, 4); fp[l] = rd(&r, fpl[l]);
    }
    uint64_t rml = rd_u(&r, 2); const uint8_t* rm = rd(&r, rml);
    uint64_t parts = rd_u(&r, 1);
    uint64_t nonce = rd_u(&r, 8);
    if (r.err || r.off != len || parts != 0) return ORC_VERIFY_FAILED;

    uint64_t seed_e[20];
    size_t ne = context_elements(n, &o, seed_e);
    memcpy(seed_e + ne, air->pub, 12 * sizeof(uint64_t));
    coin_t coin;
    coin_init(&coin, seed_e, ne + 12);
    coin_reseed(&coin, com);
    fq alpha[W], bcoef[NUM_ASSERT], z, dc[W], gam;
    for (int i = 0; i < W; i++) if (coin_draw_fq(&coin, &alpha[i])) return ORC_VERIFY_FAILED;
    for (int i = 0; i < NUM_ASSERT; i++) if (coin_draw_fq(&coin, &bcoef[i])) return ORC_VERIFY_FAILED;
    coin_reseed(&coin, com + 32);
    if (coin_draw_fq(&coin, &z)) return ORC_VERIFY_FAILED;
    fq ood[2 * W], hz = rd_fq(oe), zg = fq_mulb(z, g);
    for (int c = 0; c < 2 * W; c++) ood[c] = rd_fq(os + 1 + 16 * c);
    {
        fq cur[W], nxt[W], rr[W];
        uint64_t acol[NUM_ASSERT], astep[NUM_ASSERT], aval[NUM_ASSERT];
        for (int c = 0; c < W; c++) { cur[c] = ood[2 * c]; nxt[c] = ood[2 * c + 1]; }
        air_transition_q(air, cur, nxt, rr);
        fq t = fq_make(0, 0);
        for (int c = 0; c < W; c++) t = fq_add(t, fq_mul(alpha[c], rr[c]));
        uint64_t g_last = orc_pow(g, n - 1);
        fq zn = fq_make(1, 0);
        { fq b = z; uint64_t e = n; while (e) { if (e & 1) zn = fq_mul(zn, b); b = fq_mul(b, b); e >>= 1; } }
        fq e = fq_mul(fq_mul(t, fq_sub(z, fq_make(g_last, 0))), fq_inv(fq_sub(zn, fq_make(1, 0))));
        air_assertions(air, n, acol, astep, aval);
        fq b0 = fq_make(0, 0), b1 = fq_make(0, 0);
        for (int a = 0; a < NUM_ASSERT; a++) {
            fq term = fq_mul(bcoef[a], fq_sub(cur[acol[a]], fq_make(aval[a], 0)));
            if (astep[a] == 0) b0 = fq_add(b0, term); else b1 = fq_add(b1, term);
        }
        e = fq_add(e, fq_mul(b0, fq_inv(fq_sub(z, fq_make(1, 0)))));
        e = fq_add(e, fq_mul(b1, fq_inv(fq_sub(z, fq_make(g_last, 0)))));
        if (!fq_eq(e, hz)) return ORC_VERIFY_FAILED;
    }
    uint8_t dtmp[32];
    hash_fq(ood, 2 * W, dtmp);
    coin_reseed(&coin, dtmp);
    hash_fq(&hz, 1, dtmp);
    coin_reseed(&coin, dtmp);
    for (int c = 0; c < W; c++) if (coin_draw_fq(&coin, &dc[c])) return ORC_VERIFY_FAILED;
    if (coin_draw_fq(&coin, &gam)) return ORC_VERIFY_FAILED;
    fq falpha[16];
    for (uint32_t l = 0; l <= nl; l++) {
        coin_reseed(&coin, com + 64 + 32 * l);
        fq a;
        if (coin_draw_fq(&coin, &a)) return ORC_VERIFY_FAILED;
        if (l < nl) falpha[l] = a;
    }
    {
        uint8_t h[32];
        merge_int(coin.seed, nonce, h);
        if (tz64(get_le64(h)) < o.grinding) return ORC_VERIFY_FAILED;
    }
    coin_reseed_int(&coin, nonce);
    uint64_t pos[256], q = o.num_queries;
    for (uint64_t i = 0; i < q; i++) { uint8_t h[32]; coin_next(&coin, h); pos[i] = get_le64(h) & (N - 1); }
    qsort(pos, q, sizeof(uint64_t), cmp_u64);
    uint64_t u = 0;
    for (uint64_t i = 0; i < q; i++) if (u == 0 || pos[u - 1] != pos[i]) pos[u++] = pos[i];
    if (u != nu) return ORC_VERIFY_FAILED;

    int ok = 1;
    dg* ld = (dg*)malloc(256 * sizeof(dg));
    uint8_t root[32];
    for (uint64_t i = 0; i < nu; i++) orc_blake3(tv + i * W * 8, W * 8, ld[i]);
    if (batch_root(tp, tpl, pos, nu, ld, depth, root) || memcmp(root, com, 32)) ok = 0;
    for (uint64_t i = 0; i < nu; i++) orc_blake3(cv + i * 16, 16, ld[i]);
    if (ok && (batch_root(cp, cpl, pos, nu, ld, depth, root) || memcmp(root, com + 32, 32))) ok = 0;
    fq ev[256];
    const uint64_t wN = orc_root((unsigned)depth);
    for (uint64_t i = 0; i < nu && ok; i++) {
        uint64_t xb = orc_mul(ORC_GEN, orc_pow(wN, pos[i]));
        fq xq = fq_make(xb, 0), s1 = fq_make(0, 0), s2 = fq_make(0, 0);
        for (int c = 0; c < W; c++) {
            fq tx = fq_make(get_le64(tv + (i * W + c) * 8), 0);
            s1 = fq_add(s1, fq_mul(dc[c], fq_sub(tx, ood[2 * c])));
            s2 = fq_add(s2, fq_mul(dc[c], fq_sub(tx, ood[2 * c + 1])));
        }
        fq hx = rd_fq(cv + i * 16);
        fq izx = fq_inv(fq_sub(xq, z));
        ev[i] = fq_add(fq_mul(s1, izx), fq_mul(s2, fq_inv(fq_sub(xq, zg))));
        ev[i] = fq_add(ev[i], fq_mul(fq_mul(gam, fq_sub(hx, hz)), izx));
    }
    uint64_t D = N, cp_pos[256], ck = nu;
    memcpy(cp_pos, pos, nu * sizeof(uint64_t));
    for (uint32_t l = 0; l < nl && ok; l++) {
        uint64_t rows = D / f, np[256], nk;
        fold_positions(cp_pos, ck, rows, np, &nk);
        if (fvl[l] != nk * f * 16) { ok = 0; break; }
        for (uint64_t i = 0; i < nk; i++) orc_blake3(fv[l] + i * f * 16, f * 16, ld[i]);
        if (batch_root(fp[l], fpl[l], np, nk, ld, ilog2u(rows), root) || memcmp(root, com + 64 + 32 * l, 32)) { ok = 0; break; }
        for (uint64_t i = 0; i < ck; i++) {
            uint64_t ri = cp_pos[i] % rows, e = cp_pos[i] / rows, idx = 0;
            while (np[idx] != ri) idx++;
            if (!fq_eq(rd_fq(fv[l] + (idx * f + e) * 16), ev[i])) { ok = 0; break; }
        }
        const uint64_t wD = orc_root(ilog2u(D));
        for (uint64_t i = 0; i < nk && ok; i++) {
            fq v[16];
            for (uint64_t k = 0; k < f; k++) v[k] = rd_fq(fv[l] + (i * f + k) * 16);
            ev[i] = fri_fold_row_q(v, (uint32_t)f, orc_mul(ORC_GEN, orc_pow(wD, np[i])), falpha[l]);
        }
        memcpy(cp_pos, np, nk * sizeof(uint64_t));
        ck = nk;
        D = rows;
    }
    if (ok) {
        uint64_t rl = rml / 16;
        fq* remc = (fq*)malloc((rl + 1) * sizeof(fq));
        if (rml % 16 || rl == 0 || rl != D / beta) ok = 0;
        for (uint64_t i = 0; ok && i < rl; i++) remc[i] = rd_fq(rm + 16 * i);
        if (ok) { hash_fq(remc, rl, dtmp); if (memcmp(dtmp, com + 64 + 32 * nl, 32)) ok = 0; }
        const uint64_t wD = orc_root(ilog2u(D));
        for (uint64_t i = 0; ok && i < ck; i++)
            if (!fq_eq(horner_q(remc, rl, fq_make(orc_mul(ORC_GEN, orc_pow(wD, cp_pos[i])), 0)), ev[i])) ok = 0;
        free(remc);
    }
    free(ld);
    return ok ? ORC_OK : ORC_VERIFY_FAILED;
}
