// Proof parsing and verification state shared by the host verifier (verifier.cpp) and the batched
// GPU verifier (verify_kernels.hip + xfg_verify_batch_gpu in prover.hip).
#pragma once
#include <string>
#include <vector>

#include "host_common.hpp"
#include "kernels.hpp"

namespace xfg {

struct Span {  // bytes inside the proof
    const uint8_t* p = nullptr;
    size_t n = 0;
    u64 elem(size_t i) const {
        u64 v;
        memcpy(&v, p + 8 * i, 8);
        return v;
    }
};
// BatchMerkleProof::serialize_nodes: u8 vector count, then per vector u8 count + digests (kept as
// pointers into the proof bytes)
struct Paths {
    std::vector<const uint8_t*> ptr;
    std::vector<uint32_t> cnt;
};

// StarkProof fields in wire order (DESIGN.md "Proof format")
struct ParsedProof {
    const uint8_t* base = nullptr;  // the proof bytes every Span / Paths pointer points into
    u64 width = 0, aux = 0, logn = 0;
    Opts o{};
    u64 num_unique = 0;
    std::vector<Digest> com;  // trace root, constraint root, FRI layer roots, remainder commitment
    Span trace_rows, constraint_rows, ood, hz, fri_rem;
    Paths trace_paths, constraint_paths;
    std::vector<Span> fri_vals;
    std::vector<Paths> fri_paths;
    u64 partitions = 0, nonce = 0;
    size_t size = 0;
};
// "" on success, else the ProofDeserializationError text
std::string parse_proof(const uint8_t* bytes, size_t len, ParsedProof& pf);

// everything the query checks need, after the transcript has been replayed
struct VState {
    ParsedProof pf;
    int de = 1;  // extension degree of E
    u64 n = 0, N = 0, beta = 0;
    unsigned nl = 0;
    std::vector<u64> pos;  // unique query positions (sorted)
    E2 z{}, zg{}, hz{}, ood[14]{}, dc[7]{}, gam{};
    std::vector<E2> falpha;
};
// parse, option checks, transcript replay, OOD consistency, proof of work, query positions:
// "" when the proof may proceed to the query checks, else the VerifierError
std::string verify_transcript(const uint8_t* bytes, size_t len, const AirConst& air, const Opts& acceptable,
                              VState& st);
// the query checks on the host (Merkle openings, DEEP, FRI, remainder)
std::string verify_queries_host(const VState& st);

// symbolic BatchMerkleProof::get_root over local digest slots: slots of the queried leaves, the
// digests the proof provides, and the merges level by level (out, left, right); false when the node
// vectors do not fit the opening plan
struct MerkleSym {
    uint32_t nslots = 0, root = 0;
    std::vector<uint32_t> leaf_slot;                         // per queried leaf
    std::vector<std::pair<uint32_t, const uint8_t*>> given;  // slot, digest bytes in the proof
    std::vector<std::vector<uint32_t>> levels;               // per level: out, left, right slots
    unsigned nlev = 0;                                       // levels in use (levels may hold more)
};
bool merkle_symbolic(const std::vector<u64>& idx, const Paths& paths, u64 L, MerkleSym& out);

AirConst air_of(const xfg_air_consts* a);

}  // namespace xfg

namespace xfg {

// ---- batched GPU verification: the host replays every transcript, then the Merkle openings
// (leaf hashes + level-by-level merges over all proofs at once) and the per-query DEEP / FRI /
// remainder checks run on the device.
constexpr int VMAXL = 12;  // FRI layers
struct VLeaf {
    u64 src;          // byte offset in the proof blob
    uint32_t words;   // u64 words hashed (1, 2, 7, 8 or 16)
    uint32_t dst;     // digest slot
};
struct VGather {
    u64 src;
    uint32_t dst, pad;
};
struct VFieldProof {
    E2 z, zg, hz, gam, dc[7], ood[14];
    E2 falpha[VMAXL];
    u64 rem_off;
    uint32_t rem_len, nl, de, logN;
};
struct VFieldQuery {
    uint32_t proof, pad;
    u64 pos, trace_off, cons_off;
    u64 row_off[VMAXL];  // layer l: blob offset of the opened row of 8 E values
};
struct VerifyPlan {
    std::vector<uint8_t> blob;                 // all proofs back to back
    std::vector<VGather> gathers;
    std::vector<VLeaf> leaves;
    std::vector<std::vector<uint32_t>> rounds; // per Merkle level: (out, left, right) slot triples
    std::vector<VFieldProof> fproofs;
    std::vector<VFieldQuery> fqueries;
    uint32_t nslots = 0;
    // per proof: root slots of its 2 + nl trees in check order (-1 = structurally invalid)
    std::vector<std::vector<int64_t>> roots;
    std::vector<int> fidx;                     // proof -> index into fproofs (-1: not planned)
};
// add one proof whose transcript replayed fine; false (+ err) on a structural error
bool plan_proof(const VState& st, size_t blob_off, VerifyPlan& plan, std::string& err);
// empty a plan for reuse, keeping its allocations
void reset_plan(VerifyPlan& plan);
// the host part after the device work: first failing check in the verifier's order, "" if none
std::string finish_proof(const VState& st, const std::vector<Digest>& roots, uint32_t flags);

void launch_verify(const uint8_t* blob, const VGather* g, u64 ng, const VLeaf* lv, u64 nleaf,
                   const uint32_t* rounds, const u64* round_off, int nrounds, const VFieldProof* fp,
                   const VFieldQuery* fq, u64 nq, Digest* dig, uint32_t* flags, hipStream_t s);

}  // namespace xfg
