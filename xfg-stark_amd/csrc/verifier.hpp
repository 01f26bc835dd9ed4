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
    const uint8_t* com_p = nullptr;  // the commitments' bytes in the proof
    Span trace_rows, constraint_rows, ood, hz, fri_rem;
    Span trace_paths_raw, constraint_paths_raw, ood_raw;  // byte vectors as StarkProof::read_from keeps them
    std::vector<Span> fri_vals, fri_paths_raw;
    // filled by parse_contents
    Paths trace_paths, constraint_paths;
    std::vector<Paths> fri_paths;
    u64 partitions = 0, nonce = 0;
    size_t size = 0;
};
// StarkProof::from_bytes, structural: "" on success, else the ProofDeserializationError text
std::string parse_proof(const uint8_t* bytes, size_t len, ParsedProof& pf);
// the sections' contents (VerifierChannel::new, after the options check)
std::string parse_contents(ParsedProof& pf);

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

// ---- batched GPU verification: the host replays every transcript and lists, per proof, its 2 + nl
// batch Merkle openings and its queries; the device then verifies every opening with one workgroup
// (leaf hashes, BatchMerkleProof::get_root level by level, root comparison: vtree_kernel) and runs
// the per-query DEEP / FRI / remainder checks (vfield_kernel).
constexpr int VMAXL = 12;  // FRI layers
// flags[proof] bits set by the device: 0..11 FRI layer l folding, 16..27 FRI layer l commitment,
// 29 constraint commitment, 30 trace commitment, 31 remainder folding
constexpr uint32_t VF_TRACE = 1u << 30, VF_CONSTRAINT = 1u << 29, VF_REMAINDER = 1u << 31;
constexpr int VF_LAYER_COMMIT = 16;
struct VTree {
    u64 root_off;           // blob offset of the commitment the root must equal
    uint32_t leaf0, nidx;   // opened leaves: tleaves[leaf0 .. leaf0 + nidx), sorted by index
    uint32_t vec0, nvec;    // node vectors: vecs[vec0 .. vec0 + nvec), in the proof's order
    uint32_t words, depth;  // u64 words per leaf (1, 2, 7, 8 or 16); log2 leaves
    uint32_t proof, bit;    // on failure: flags[proof] |= bit
};
struct VTreeLeaf {
    u64 index;    // leaf index
    u64 row_off;  // blob offset of the opened row
};
struct VVec {
    u64 off;  // blob offset of the vector's first digest
    uint32_t cnt, pad;
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
// one proof's part of a batch (blob offsets already global; tree / vector / proof indices local)
struct VerifyPlan {
    std::vector<VTree> trees;
    std::vector<VTreeLeaf> tleaves;
    std::vector<VVec> vecs;
    VFieldProof fproof{};
    std::vector<VFieldQuery> fqueries;
};
// plan one proof whose transcript replayed fine, its bytes at blob offset blob_off; false (+ err) on
// a structural error the host verifier reports before any opening is checked
bool plan_proof(const VState& st, size_t blob_off, VerifyPlan& plan, std::string& err);
// the host part after the device work: first failing check in the verifier's order, "" if none
std::string finish_proof(const VState& st, uint32_t flags);

void launch_verify(const uint8_t* blob, const VTree* trees, u64 ntrees, const VTreeLeaf* tleaves, const VVec* vecs,
                   const VFieldProof* fp, const VFieldQuery* fq, u64 nq, uint32_t* flags, hipStream_t s);

}  // namespace xfg
