/*
 * ORACLE / TEST INFRASTRUCTURE ONLY. Loaded only by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg; the product never links it.
 *
 * CPU restatement (single-threaded plain C) of the XFG burn-proof STARK path:
 *   reference  src/burn_mint_prover.rs:62-129   XfgBurnMintProver::prove_burn_mint
 *              src/burn_mint_air.rs:124-202      Keccak-derived AIR constants
 *              src/burn_mint_air.rs:335-395      transition constraints + assertions
 *              src/burn_mint_air.rs:442-476      trace
 *              src/burn_mint_air.rs:479-531      Prover binding (Blake3_256, DefaultRandomCoin,
 *                                                DefaultTraceLde, DefaultConstraintEvaluator)
 *   + the Winterfell 0.8.3 proving pipeline the reference calls (air.prove, :124-126), which is an
 *     external crate not present in /root/reference. Its algorithm is restated from the published
 *     Winterfell 0.8 design -- every such step is marked RECALLED in
 *     orc_stark.c.
 *
 * PARITY STATUS: primitives (field, BLAKE3, Keccak-256, AIR constants, marshalling) are pinned
 * by the reference's own KATs and the published hash test vectors. Whole-proof bytes are
 * "parity unpinned" against real Winterfell: the reference cannot be built here (no Rust
 * toolchain) and its prove_burn_mint panics for every input; no reference test
 * holds proof bytes. The corrected-AIR contract is SURVEY.md Appendix A.
 */
#ifndef XFG_ORACLE_H
#define XFG_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t num_queries;      /* 42 in the reference */
    uint32_t blowup;           /* 8 */
    uint32_t grinding;         /* 4 */
    uint32_t field_extension;  /* 1 = None (Winterfell FieldExtension::None) */
    uint32_t fri_folding;      /* 8 */
    uint32_t fri_rem_max_deg;  /* 31 */
} orc_options;

/* AIR instance: 12 public-input elements (BurnMintPublicInputs::to_elements order,
 * reference src/burn_mint_air.rs:54-71), the secret element and the two Keccak constants. */
typedef struct {
    uint64_t pub[12];
    uint64_t secret;
    uint64_t nullifier;
    uint64_t commitment;
} orc_air;

/* intermediate values exposed for stage-by-stage GPU parity debugging */
typedef struct {
    uint8_t trace_root[32];
    uint8_t constraint_root[32];
    uint8_t fri_roots[16][32];
    uint32_t num_fri_layers;
    uint64_t z;
    uint64_t ood[15];
    uint64_t pow_nonce;
    uint32_t num_unique_queries;
    uint64_t positions[256];
} orc_debug;

enum {
    ORC_OK = 0,
    ORC_INVALID_BURN_AMOUNT = 1,
    ORC_MINT_MISMATCH = 2,
    ORC_ZERO_TX_HASH = 3,
    ORC_BAD_RECIPIENT_LEN = 4,
    ORC_SHORT_SECRET = 5,
    ORC_PROVER_ERROR = 6,
    ORC_BUFFER_TOO_SMALL = 8,
    ORC_VERIFY_FAILED = 9,
};

/* input validation + marshalling (src/burn_mint_prover.rs:62-118,132-221) + AIR constants
 * (src/burn_mint_air.rs:124-202). Returns ORC_OK or a validation status. */
int orc_burn_air_from_inputs(uint64_t burn_amount, uint64_t mint_amount, const uint8_t tx_prefix_hash[32],
                             const uint8_t* recipient, size_t recipient_len, const uint8_t* secret,
                             size_t secret_len, uint32_t network_id, uint32_t target_chain_id,
                             uint32_t commitment_version, orc_air* out);
/* Keccak constants from (pub, secret): nullifier, recipient_full(32B), commitment */
void orc_air_constants(const uint64_t pub[12], uint64_t secret, uint64_t* nullifier, uint8_t recipient_full[32],
                       uint64_t* commitment);
/* length-generic burn trace, column-major [7][n] */
void orc_build_trace(const orc_air* air, uint64_t n, uint64_t* trace);

/* prove over an execution trace. faithful != 0 recomputes the three Keccak constants for every
 * constraint-evaluation row exactly as the reference does (src/burn_mint_air.rs:264,376); the
 * proof bytes are identical either way. out == NULL -> *out_len = required size. */
int orc_prove(const orc_air* air, const uint64_t* trace, uint64_t n, const orc_options* opt, int faithful,
              uint8_t* out, size_t* out_len, orc_debug* dbg);
/* `count` proofs over `threads` OpenMP threads (bench.py's CPU baseline: 1 thread faithful, and all
 * cores); stage_ms[ORC_NSTAGE] = summed CPU ms per stage: trace LDE, trace commitment, constraint
 * evaluation, composition (+ commitment), OOD + DEEP, FRI, grinding + queries, serialisation.
 * Returns the number of threads that ran. */
#define ORC_NSTAGE 8
int orc_prove_batch(const orc_air* airs, uint32_t count, uint64_t n, const orc_options* opt, int faithful,
                    int threads, size_t* lens, int* statuses, double* stage_ms);
/* evaluate_transition on one frame (src/burn_mint_air.rs:335-378) */
void orc_eval_transition(const orc_air* air, const uint64_t cur[7], const uint64_t nxt[7], uint64_t r[7]);
/* upper bound on proof size for buffer allocation */
size_t orc_proof_size_bound(uint64_t n, const orc_options* opt);
/* verifier restatement (Winterfell 0.8 verify) used as the oracle's self-check */
int orc_verify(const orc_air* air, const uint8_t* proof, size_t len, const orc_options* opt);

/* primitives exported for KAT tests */
void orc_blake3_bytes(const uint8_t* in, size_t len, uint8_t out[32]);
void orc_keccak256_bytes(const uint8_t* in, size_t len, uint8_t out[32]);
void orc_sha3_256_bytes(const uint8_t* in, size_t len, uint8_t out[32]);
uint64_t orc_field_mul(uint64_t a, uint64_t b);
uint64_t orc_field_root(uint32_t k);
/* natural-order NTT helpers (coefficients <-> evaluations) for kernel-level parity tests */
void orc_interpolate(uint64_t* vals, uint64_t n, uint64_t offset);                       /* in place */
void orc_evaluate_lde(const uint64_t* coef, uint64_t n, uint64_t blowup, uint64_t offset, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
