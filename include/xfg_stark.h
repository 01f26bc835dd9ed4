/*
 * xfg_stark.h -- C ABI of the MI355X-native XFG burn-proof STARK prover (libxfgstark.so).
 *
 * Drop-in boundary for the reference's proving path. Rust is not available in this build
 * environment, so the host side above this ABI is C++ (inside the .so) and the reference-side
 * binding a Rust maintainer would add is shown in INTEGRATION.md. Every entry point replaces a
 * reference interface:
 *
 *   xfg_prove_burn_mint  <- XfgBurnMintProver::prove_burn_mint      src/burn_mint_prover.rs:62-129
 *                           (validate_inputs :132-180, secret_to_field_element :195-208,
 *                            compute_recipient_hash :211-221, air.prove(trace) :124-126)
 *   xfg_prove_trace      <- <XfgBurnMintAir as winterfell::Prover>::prove(trace)
 *                           src/burn_mint_air.rs:479-531 (ExecutionTrace-level entry; trace layout
 *                           of build_trace :442-476, column-major)
 *   xfg_prove_batch      <- the serial loops of the reference callers (e.g. benchmark harness
 *                           src/benchmarks/mod.rs:301-342, BatchBurnMintVerifier's pattern
 *                           src/burn_mint_verifier.rs:326-338) -- independent proofs, one launch set
 *   xfg_default_options  <- XfgBurnMintProver::new(_) ProofOptions::new(42, 8, 4, None, 8, 31)
 *                           src/burn_mint_prover.rs:27-41 (argument order: queries, blowup,
 *                           grinding, extension, FRI folding, FRI remainder max degree)
 *   xfg_proof_size_bound <- XfgBurnMintProver::get_proof_size  src/burn_mint_prover.rs:224-227
 *   xfg_last_error       <- XfgStarkError::CryptoError(String) text  src/burn_mint_prover.rs:143-177
 *
 * Output bytes are the proof's `StarkProof::to_bytes()` serialisation as restated in DESIGN.md
 * ("Proof format"); the caller owns all host buffers, the library owns device memory (pooled per
 * context). `out == NULL` (or *out_len too small) returns the required size in *out_len.
 * A context is bound to one HIP device; it owns XFG_LANES (default 7) lanes, each a HIP stream with
 * its workspace and a host worker thread; the per-proof host work of the lanes (transcript replay,
 * opening plans, serialisation) runs on a process-wide pool of XFG_HOST_THREADS (default 8) threads.
 * Submit from one thread per context.
 */
#ifndef XFG_STARK_H
#define XFG_STARK_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct xfg_ctx xfg_ctx;

typedef enum {
    XFG_OK = 0,
    XFG_INVALID_BURN_AMOUNT = 1, /* burn not 8,000,000 or 8,000,000,000 atomic units */
    XFG_MINT_MISMATCH = 2,       /* mint != burn (1:1) */
    XFG_ZERO_TX_HASH = 3,        /* u64 LE of tx_prefix_hash[0..8] == 0 */
    XFG_BAD_RECIPIENT_LEN = 4,   /* recipient address not 20 bytes */
    XFG_SHORT_SECRET = 5,        /* secret shorter than 8 bytes (reference: error <4, panic 4..7) */
    XFG_PROVER_ERROR = 6,        /* Winterfell prover error / unsupported options */
    XFG_DEVICE_ERROR = 7,        /* HIP runtime failure */
    XFG_BUFFER_TOO_SMALL = 8,
    XFG_INVALID_ARGUMENT = 9,
    XFG_VERIFY_FAILED = 10       /* proof rejected (verifier) or not a well-formed proof (parser) */
} xfg_status;

/* winterfell::ProofOptions (0.8) */
typedef struct {
    uint32_t num_queries;
    uint32_t blowup_factor;
    uint32_t grinding_factor;
    uint32_t field_extension; /* 1 = FieldExtension::None */
    uint32_t fri_folding_factor;
    uint32_t fri_remainder_max_degree;
} xfg_options;

/* arguments of prove_burn_mint (src/burn_mint_prover.rs:62-72) */
typedef struct {
    uint64_t burn_amount;
    uint64_t mint_amount;
    uint8_t tx_prefix_hash[32];
    const uint8_t* recipient_address;
    size_t recipient_len;
    const uint8_t* secret;
    size_t secret_len;
    uint32_t network_id;
    uint32_t target_chain_id;
    uint32_t commitment_version;
} xfg_burn_inputs;

/* AIR instance for ExecutionTrace-level proving: BurnMintPublicInputs::to_elements
 * (src/burn_mint_air.rs:54-71) + the two Keccak-derived constants (:124-133, :174-202) */
typedef struct {
    uint64_t pub_inputs[12];
    uint64_t nullifier;
    uint64_t commitment;
} xfg_air_consts;

xfg_ctx* xfg_ctx_create(int device_id);
void xfg_ctx_destroy(xfg_ctx* ctx);
int xfg_default_options(xfg_options* out);
/* length of the error text of the last failing call on ctx (copied NUL-terminated into buf) */
int xfg_last_error(const xfg_ctx* ctx, char* buf, size_t len);
/* the largest proof the prover emits for (trace_length, opts): a tight upper bound computed section
 * by section (every proof fits; configs[2]: 98.8 KB for ~78 KB proofs), so callers can size fixed
 * per-proof output slots, e.g. the exchange records of a sharded run; 0 for unsupported shapes */
size_t xfg_proof_size_bound(uint64_t trace_length, const xfg_options* opts);

/* prove_burn_mint; trace_length 0 -> 64 (the reference's fixed TraceInfo::new(7, 64)) */
int xfg_prove_burn_mint(xfg_ctx* ctx, const xfg_burn_inputs* in, uint64_t trace_length, const xfg_options* opts,
                        uint8_t* out, size_t* out_len);
/* prove over a caller-supplied execution trace, column-major [width][n], width must be 7 */
int xfg_prove_trace(xfg_ctx* ctx, const uint64_t* trace, uint32_t width, uint64_t n, const xfg_air_consts* air,
                    const xfg_options* opts, uint8_t* out, size_t* out_len);
/* batch of independent proofs on this context's device; statuses[i] per proof, returns XFG_OK if
 * the batch ran (individual proofs may still carry validation errors) */
int xfg_prove_batch(xfg_ctx* ctx, uint32_t count, const xfg_burn_inputs* inputs, uint64_t trace_length,
                    const xfg_options* opts, uint8_t* const* outs, size_t* out_lens, int* statuses);

/* asynchronous form of xfg_prove_batch for pipelined callers (a proving service, bench.py):
 * inputs are validated and marshalled before this returns (statuses[i] of invalid inputs are set
 * now); outs / out_lens / statuses must stay valid until xfg_batch_wait(ticket) returns. Batches
 * submitted back to back share the context's lane workers, so the host-side tail of one (query
 * openings, serialisation) overlaps the kernels of the next. */
int xfg_prove_batch_submit(xfg_ctx* ctx, uint32_t count, const xfg_burn_inputs* inputs, uint64_t trace_length,
                           const xfg_options* opts, uint8_t* const* outs, size_t* out_lens, int* statuses,
                           uint64_t* ticket);
/* blocks until the batch is proven and its outputs written; returns like xfg_prove_batch */
int xfg_batch_wait(xfg_ctx* ctx, uint64_t ticket);

/* allocate every device / pinned-host workspace and load all code objects for batches of
 * `count` proofs of this shape (setup, not a prove; later calls never allocate) */
int xfg_prepare(xfg_ctx* ctx, uint32_t count, uint64_t trace_length, const xfg_options* opts);

/* AIR constants from raw inputs (marshalling + Keccak, host); returns a validation status */
int xfg_burn_air_consts(const xfg_burn_inputs* in, xfg_air_consts* out);

/* ---- proofs: parsing and verification (host; no device needed) ---- */
/* header of a parsed proof (StarkProof::from_bytes, winter-air 0.8) */
typedef struct {
    uint32_t trace_width;
    uint64_t trace_length;
    xfg_options options;
    uint32_t num_unique_queries;
    uint32_t num_fri_layers;
    uint32_t remainder_len;     /* FRI remainder coefficients (E elements, not coordinates) */
    uint64_t pow_nonce;
    uint8_t trace_root[32];
    uint8_t constraint_root[32];
    uint64_t ood_trace[14];     /* T_c(z), T_c(z g) interleaved (first coordinates with an extension) */
    uint64_t ood_composition;   /* H(z) */
    size_t size;                /* bytes consumed == len for a well-formed proof */
} xfg_proof_info;

/* StarkProof::from_bytes <- src/burn_mint_prover.rs:224-227 (to_bytes), src/bin/xfg-stark-cli.rs:533-558
 * structural parse of proof bytes; XFG_VERIFY_FAILED + ProofDeserializationError text on bad input */
int xfg_proof_parse(const uint8_t* proof, size_t len, xfg_proof_info* info, char* err, size_t err_len);

/* winterfell::verify::<XfgBurnMintAir, Blake3_256, DefaultRandomCoin> with
 * AcceptableOptions::OptionSet([*acceptable])  <- XfgBurnMintVerifier::verify_with_public_inputs /
 * verify_with_winterfell, src/burn_mint_verifier.rs:186-203, 265-283. The statement is the AIR
 * constants (12 public inputs + nullifier + commitment, see xfg_burn_air_consts). XFG_OK = accepted;
 * XFG_VERIFY_FAILED = rejected, err receives the VerifierError (Debug form, e.g.
 * "InconsistentOodConstraintEvaluations"). */
int xfg_verify(const uint8_t* proof, size_t len, const xfg_air_consts* air, const xfg_options* acceptable, char* err,
               size_t err_len);
/* BatchBurnMintVerifier::verify_batch <- src/burn_mint_verifier.rs:386-408 (and batch_verify
 * :326-338): results[i] = xfg_verify status of proof i; `threads` host threads (0 = all cores) */
int xfg_verify_batch(uint32_t count, const uint8_t* const* proofs, const size_t* lens, const xfg_air_consts* airs,
                     const xfg_options* acceptable, int* results, uint32_t threads);

/* batched verification on the context's GPU: the host replays each transcript (threads), the device
 * recomputes every Merkle opening (leaf hashes, then one launch per tree level for all proofs) and
 * runs the per-query DEEP / FRI / remainder checks. results[i] as xfg_verify. */
int xfg_verify_batch_gpu(xfg_ctx* ctx, uint32_t count, const uint8_t* const* proofs, const size_t* lens,
                         const xfg_air_consts* airs, const xfg_options* acceptable, int* results);

/* ---- instrumentation (benchmarks / parity tests) ---- */
/* host BLAKE3 of the library (any length), for self-tests */
int xfg_selftest_blake3(const uint8_t* in, size_t len, uint8_t out[32]);
/* host-side field arithmetic of the library (mul, add, sub) for self-tests; canonical inputs */
int xfg_selftest_field(uint64_t a, uint64_t b, uint64_t* out3);
/* per-stage device milliseconds of the last prove call when timing is enabled (returns count) */
int xfg_set_timing(xfg_ctx* ctx, int enabled);
int xfg_stage_times(const xfg_ctx* ctx, double* ms, const char** names, int max);
/* times `iters` launches of the trace LDE kernels (7 columns x count proofs, resident device
 * buffers, HIP events on the context stream); returns average ms per launch set in *avg_ms */
int xfg_bench_lde(xfg_ctx* ctx, uint32_t count, uint64_t n, uint32_t blowup, uint32_t iters, double* avg_ms);
/* in-pipeline trace-LDE timing: HIP events around the trace LDE launch set of every proof unit
 * (on the lane stream that launches it). enabled = 1 resets and starts; enabled = 0 stops. The
 * totals so far (sum of launch-set durations, launch sets, polynomials) are returned either way. */
int xfg_lde_probe(xfg_ctx* ctx, int enabled, double* total_ms, uint64_t* launch_sets, uint64_t* polys);
/* kernel-level parity hooks (host buffers in/out) */
int xfg_debug_lde(xfg_ctx* ctx, const uint64_t* coef, uint32_t npoly, uint64_t n, uint32_t blowup, uint64_t* out);
int xfg_debug_interpolate(xfg_ctx* ctx, const uint64_t* evals, uint32_t npoly, uint64_t n, int offset7,
                          uint64_t* out);
/* Goldilocks primitive self test on the device: out[i] = op(a[i], b[i]) with op 0 mul, 1 add,
 * 2 sub, 3 canonical(a), 4 a * 2^(b mod 96), 5 a + (b mod 2^32) * (2^32 - 1), 6 a - b with one
 * borrow fold (the weak subtraction of the NTT butterflies), 7 a + b with one carry fold (the weak
 * addition of the NTT butterflies, b < p), 8 a * b through the interleaved pair multiply (gl_mul2:
 * both a * b and b * a computed, all ones returned if they differ) */
int xfg_debug_field(xfg_ctx* ctx, uint32_t op, uint64_t count, const uint64_t* a, const uint64_t* b, uint64_t* out);
/* OOD evaluation + DEEP quotient kernels of the prover on `count` instances: coef [count][7][n],
 * hcoef [count][n] (trace / composition coefficients), zpts [count][2] = (z, z g), coeffs
 * [count][8] = 7 trace DEEP coefficients + the composition one; ood_out [count][15] (T_c(z),
 * T_c(zg) interleaved, H(z)), deep_out [count][n] (DEEP composition coefficients) */
int xfg_debug_ood_deep(xfg_ctx* ctx, uint32_t count, uint64_t n, const uint64_t* coef, const uint64_t* hcoef,
                       const uint64_t* zpts, const uint64_t* coeffs, uint64_t* ood_out, uint64_t* deep_out);
/* device Fiat-Shamir draws (DefaultRandomCoin<Blake3_256>::draw::<E>) from the coin (seed as 8 LE
 * u32 words, counter): k <= 64 draws of E (ext 1 or 2) by one wave -- the prover's coefficient and
 * DEEP draws -- and one at a time -- its FRI alpha draws. Besides the >= p rule, a candidate whose
 * counter c (1 <= c <= 256) has bit c - 1 of reject[4] set is rejected, to exercise the retries.
 * out_wave / out_seq [k][2] (second coordinate 0 when ext = 1), counters[2] = each coin's counter
 * afterwards, ok[2] = 1 when no draw ran out of its 1000 tries */
int xfg_debug_coin_draws(xfg_ctx* ctx, const uint32_t seed[8], uint64_t counter, uint32_t k, uint32_t ext,
                         const uint64_t reject[4], uint64_t* out_wave, uint64_t* out_seq, uint64_t counters[2],
                         int ok[2]);

#ifdef __cplusplus
}
#endif
#endif
