"""Product proof parser + verifier (libxfgstark.so host code, no GPU) against oracle-made proofs.

SURVEY.md §8(f) rows 1-2: StarkProof::from_bytes and winterfell::verify for the burn AIR
(src/burn_mint_verifier.rs:186-283, batch :326-408). The proofs come from the oracle (the CPU
restatement of the prover) and from the committed golden fixture, so this checks the product
verifier against an independent implementation of the same protocol; tampering each proof section
must produce the matching VerifierError."""
import json
import os
import struct

import pytest

import oracle_lib as O
import synthetic

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def X():
    import xfgstark
    return xfgstark


def _statement(X, kw):
    return X.air_consts(**kw)


def _oracle_proof(kw, n, **opts):
    st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"], kw["recipient_address"],
                                kw["secret"], kw["network_id"], kw["target_chain_id"], kw["commitment_version"])
    assert st == 0
    st, proof = O.prove(air, n, O.options(**opts))
    assert st == 0
    assert O.verify(air, proof, O.options(**opts)) == 0
    return proof


def _opts(X, **kw):
    o = X.ProofOptions.reference()
    names = {"blowup": "blowup_factor", "fri_rem_max_deg": "fri_remainder_max_degree", "grinding": "grinding_factor",
             "num_queries": "num_queries", "field_extension": "field_extension"}
    for k, v in kw.items():
        setattr(o, names[k], v)
    return o


def _sections(proof):
    """byte offsets of the proof sections (test-side walk of the wire layout)"""
    off = {}
    p = 0
    meta = struct.unpack_from("<H", proof, 3)[0]
    p = 5 + meta + 1 + 8 + 6
    p += 1  # num_unique_queries
    clen = struct.unpack_from("<H", proof, p)[0]
    off["commitments"] = p + 2
    p += 2 + clen + 1
    for name in ("trace_rows", "trace_paths", "constraint_rows", "constraint_paths"):
        ln = struct.unpack_from("<I", proof, p)[0]
        off[name] = (p + 4, ln)
        p += 4 + ln
    ln = struct.unpack_from("<H", proof, p)[0]
    off["ood"] = (p + 2 + 1, ln - 1)
    p += 2 + ln
    ln = struct.unpack_from("<H", proof, p)[0]
    off["hz"] = (p + 2, ln)
    p += 2 + ln
    nl = proof[p]
    p += 1
    for l in range(nl):
        for name in ("fri_vals", "fri_paths"):
            ln = struct.unpack_from("<I", proof, p)[0]
            off[f"{name}{l}"] = (p + 4, ln)
            p += 4 + ln
    ln = struct.unpack_from("<H", proof, p)[0]
    off["remainder"] = (p + 2, ln)
    p += 2 + ln + 1
    off["nonce"] = (p, 8)
    assert p + 8 == len(proof)
    return off


def _flip(proof, at):
    b = bytearray(proof)
    b[at] ^= 0x01
    return bytes(b)


def test_blake3_any_length_matches_oracle(X):
    for L in (0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3072, 4097, 8209):
        d = bytes((i * 131 + 7) & 255 for i in range(L))
        assert X.blake3(d) == O.blake3(d), L


def test_from_bytes_golden_fixture(X):
    case = [c for c in json.load(open(os.path.join(GOLD, "proofs.json"))) if c.get("proof_hex")][0]
    data = bytes.fromhex(case["proof_hex"])
    p = X.StarkProof.from_bytes(data)
    assert p.to_bytes() == data and len(p) == case["len"]
    assert p.trace_length == case["n"]
    o = p.options
    assert (o.num_queries, o.blowup_factor, o.grinding_factor, o.field_extension, o.fri_folding_factor,
            o.fri_remainder_max_degree) == (42, case["blowup"], 4, 1, 8, 31)
    assert 0 < p.num_unique_queries <= 42 and p.num_fri_layers >= 1
    tz, tzg, hz = p.ood_frame
    assert len(tz) == len(tzg) == 7
    assert tz[0] == synthetic.REFERENCE_PACKAGE["burn_amount"]  # constant column: T_0(z) = burn


def test_from_bytes_rejects_malformed(X):
    case = [c for c in json.load(open(os.path.join(GOLD, "proofs.json"))) if c.get("proof_hex")][0]
    data = bytes.fromhex(case["proof_hex"])
    for bad in (data[:-1], data + b"\0", data[:10], b""):
        with pytest.raises(X.XfgStarkError) as e:
            X.StarkProof.from_bytes(bad)
        assert e.value.status == 10 and "ProofDeserializationError" in str(e.value)
    # OOD frames with fewer (or more) values than 2 rows x 7 columns: from_bytes keeps the frame as a
    # byte vector (structural, as StarkProof::read_from) and reads none of its values -- the header
    # reports a zero frame (an empty frame used to be read past the end); the verifier's
    # content parse rejects the layout (after the options check)
    sec = _sections(data)
    at, ln = sec["ood"]
    for k in (0, 2, 13, 15):
        frame = (data[at:at + ln] * 2)[:8 * k]
        bad = data[:at - 3] + struct.pack("<H", 1 + 8 * k) + b"\x02" + frame + data[at + ln:]
        assert X.StarkProof.from_bytes(bad).ood_frame == ([0] * 7, [0] * 7, 0), k
        ok, err, _ = X.XfgBurnMintVerifier().verify_with_details(bad, _statement(X, synthetic.REFERENCE_PACKAGE))
        assert not ok and "OOD frame layout" in err, (k, err)
    # an invalid field extension byte in the context
    ext_at = 5 + struct.unpack_from("<H", data, 3)[0] + 1 + 8 + 3
    for ext in (0, 4, 255):
        bad = data[:ext_at] + bytes([ext]) + data[ext_at + 1:]
        with pytest.raises(X.XfgStarkError) as e:
            X.StarkProof.from_bytes(bad)
        assert "invalid field extension" in str(e.value), ext


def _set_elem(proof, at, value):
    return proof[:at] + struct.pack("<Q", value) + proof[at + 8:]


def test_noncanonical_elements_rejected(X):
    """A value >= p in any element field of the proof is a deserialization error (winter-math
    BaseElement::read_from), not arithmetic on a non-reduced operand."""
    P = 0xFFFFFFFF00000001
    kws = synthetic.burn_inputs(5)
    proof = _oracle_proof(kws, 256)
    air = _statement(X, kws)
    v = X.XfgBurnMintVerifier()
    sec = _sections(proof)
    # opened trace row, column 0 = burn amount (constant column, so its LDE value is small): v + p
    at = sec["trace_rows"][0]
    val = struct.unpack_from("<Q", proof, at)[0]
    assert val == kws["burn_amount"] and val + P < 1 << 64
    ok, err, _ = v.verify_with_details(_set_elem(proof, at, val + P), air)
    assert not ok and err == 'ProofDeserializationError("invalid field element")', err
    # the same value in the OOD frame: T_0(z) = burn for the constant column
    at = sec["ood"][0]
    assert struct.unpack_from("<Q", proof, at)[0] == kws["burn_amount"]
    ok, err, _ = v.verify_with_details(_set_elem(proof, at, kws["burn_amount"] + P), air)
    assert not ok and err == 'ProofDeserializationError("invalid field element")', err
    # >= p (no canonical preimage needed) in each other element section
    for name in ("constraint_rows", "hz", "fri_vals0", "remainder"):
        at = sec[name][0]
        bad = _set_elem(proof, at, 0xFFFFFFFFFFFFFFFF)
        ok, err, _ = v.verify_with_details(bad, air)
        assert not ok and err == 'ProofDeserializationError("invalid field element")', (name, err)
        # Proof::from_bytes keeps the element sections as raw bytes (winterfell 0.8): structural only
        assert X.StarkProof.from_bytes(bad).to_bytes() == bad
    # p itself is non-canonical too; p - 1 parses (and then fails a check, not the parser)
    at = sec["remainder"][0]
    ok, err, _ = v.verify_with_details(_set_elem(proof, at, P), air)
    assert not ok and err.startswith("ProofDeserializationError"), err
    ok, err, _ = v.verify_with_details(_set_elem(proof, at, P - 1), air)
    assert not ok and err.startswith("FriVerificationFailed"), err


def test_options_checked_before_elements(X):
    """error precedence of winterfell::verify: the acceptable-options check comes before
    VerifierChannel::new deserialises the element sections, so a proof with other
    options AND a value >= p reports UnacceptableProofOptions"""
    kws = synthetic.burn_inputs(5)
    proof = _oracle_proof(kws, 256)
    bad = _set_elem(proof, _sections(proof)["remainder"][0], 0xFFFFFFFFFFFFFFFF)
    other = X.ProofOptions.reference()
    other.num_queries = 41
    ok, err, _ = X.XfgBurnMintVerifier(proof_options=other).verify_with_details(bad, _statement(X, kws))
    assert not ok and err == "UnacceptableProofOptions", err
    ok, err, _ = X.XfgBurnMintVerifier().verify_with_details(bad, _statement(X, kws))
    assert not ok and err == 'ProofDeserializationError("invalid field element")', err


@pytest.mark.parametrize("section", ["trace_paths", "fri_paths0", "ood_layout"])
def test_options_checked_before_section_contents(X, section):
    """StarkProof::read_from keeps the Merkle paths, the OOD frame and the remainder as byte vectors;
    their contents are parsed in VerifierChannel::new, after the acceptable-options check (ADVICE
    r03). A malformed path blob or OOD frame layout with other options reports
    UnacceptableProofOptions, from_bytes accepts it, and with the right options it is a
    ProofDeserializationError. (No reference fixture covers this: parity unpinned.)"""
    kws = synthetic.burn_inputs(6)
    proof = bytearray(_oracle_proof(kws, 256))
    secs = _sections(bytes(proof))
    if section == "ood_layout":
        proof[secs["ood"][0] - 1] = 3  # frame size byte of the OOD trace states
    else:
        at, ln = secs[section]
        proof[at] ^= 0x05  # the node-vector count: the vectors no longer tile the blob
    bad = bytes(proof)
    X.StarkProof.from_bytes(bad)  # structural parse only
    other = X.ProofOptions.reference()
    other.num_queries = 41
    ok, err, _ = X.XfgBurnMintVerifier(proof_options=other).verify_with_details(bad, _statement(X, kws))
    assert not ok and err == "UnacceptableProofOptions", err
    ok, err, _ = X.XfgBurnMintVerifier().verify_with_details(bad, _statement(X, kws))
    assert not ok and err.startswith("ProofDeserializationError"), err


def test_from_bytes_remainder_len_counts_elements(X):
    for kw in (dict(), dict(field_extension=2)):
        kws = synthetic.burn_inputs(9)
        proof = _oracle_proof(kws, 256, **kw)
        p = X.StarkProof.from_bytes(proof)
        de = kw.get("field_extension", 1)
        assert p.remainder_len == _sections(proof)["remainder"][1] // (8 * de)
        # (31 + 1) coefficients at most: remainder degree bound of the reference options
        assert p.remainder_len <= 32


def test_verifier_accepts_golden_fixture(X):
    case = [c for c in json.load(open(os.path.join(GOLD, "proofs.json"))) if c.get("proof_hex")][0]
    v = X.XfgBurnMintVerifier()
    ok, err, size = v.verify_with_details(bytes.fromhex(case["proof_hex"]), _statement(X, synthetic.REFERENCE_PACKAGE))
    assert ok and err is None and size == case["len"]
    assert v.verify_burn_mint(bytes.fromhex(case["proof_hex"]), **synthetic.REFERENCE_PACKAGE)


@pytest.mark.parametrize("n,kw", [(64, dict(blowup=4)), (1024, dict()), (2048, dict(fri_rem_max_deg=255)),
                                  (256, dict(blowup=16, num_queries=24)), (512, dict(blowup=2, grinding=0)),
                                  (64, dict(field_extension=2)), (1024, dict(field_extension=2, blowup=16, num_queries=24)),
                                  (2048, dict(field_extension=2, fri_rem_max_deg=127))])
def test_verifier_accepts_oracle_proofs(X, n, kw):
    kws = synthetic.burn_inputs(n + len(kw))
    proof = _oracle_proof(kws, n, **kw)
    v = X.XfgBurnMintVerifier(proof_options=_opts(X, **kw))
    ok, err, _ = v.verify_with_details(proof, _statement(X, kws))
    assert ok, err


def test_verifier_rejects_tampering_with_reference_errors(X):
    kws = synthetic.burn_inputs(5)
    proof = _oracle_proof(kws, 256)
    air = _statement(X, kws)
    v = X.XfgBurnMintVerifier()
    sec = _sections(proof)
    expect = {
        "trace_rows": "TraceQueryDoesNotMatchCommitment",
        "constraint_rows": "ConstraintQueryDoesNotMatchCommitment",
        "ood": "InconsistentOodConstraintEvaluations",
        "hz": "InconsistentOodConstraintEvaluations",
        "fri_vals0": "FriVerificationFailed",
        "remainder": "FriVerificationFailed",
    }
    for name, want in expect.items():
        at = sec[name][0] + 3
        ok, err, _ = v.verify_with_details(_flip(proof, at), air)
        assert not ok and err.startswith(want), (name, err)
    # a digest inside the trace paths: the recomputed root differs
    ok, err, _ = v.verify_with_details(_flip(proof, sec["trace_paths"][0] + 2 + 5), air)
    assert not ok and err == "TraceQueryDoesNotMatchCommitment"
    # commitments feed the transcript: any change moves z, the OOD check fails first
    ok, err, _ = v.verify_with_details(_flip(proof, sec["commitments"] + 40), air)
    assert not ok
    # nonce: proof of work or the query positions no longer match
    ok, err, _ = v.verify_with_details(_flip(proof, sec["nonce"][0]), air)
    assert not ok
    # another statement (different nullifier) is rejected
    pub, nf, cm = air
    ok, err, _ = v.verify_with_details(proof, (pub, nf ^ 1, cm))
    assert not ok and err == "InconsistentOodConstraintEvaluations"
    # options outside the acceptable set
    ok, err, _ = X.XfgBurnMintVerifier(proof_options=_opts(X, num_queries=41)).verify_with_details(proof, air)
    assert not ok and err == "UnacceptableProofOptions"


def test_verifier_quadratic_tampering(X):
    """FieldExtension::Quadratic proofs (E-valued OOD frame, composition rows, FRI layers)"""
    kws = synthetic.burn_inputs(77)
    kw = dict(field_extension=2)
    proof = _oracle_proof(kws, 256, **kw)
    air = _statement(X, kws)
    v = X.XfgBurnMintVerifier(proof_options=_opts(X, **kw))
    assert v.verify_with_public_inputs(proof, air)
    sec = _sections(proof)
    for name, want in {"constraint_rows": "ConstraintQueryDoesNotMatchCommitment",
                       "ood": "InconsistentOodConstraintEvaluations", "hz": "InconsistentOodConstraintEvaluations",
                       "fri_vals0": "FriVerificationFailed", "remainder": "FriVerificationFailed"}.items():
        for at in (sec[name][0] + 1, sec[name][0] + 9):  # first and second coordinate of an element
            ok, err, _ = v.verify_with_details(_flip(proof, at), air)
            assert not ok and err.startswith(want), (name, at, err)
    # the same proof is not acceptable as a base-field proof and vice versa
    assert not X.XfgBurnMintVerifier().verify_with_public_inputs(proof, air)
    p = X.StarkProof.from_bytes(proof)
    assert p.options.field_extension == 2 and p.trace_length == 256


def test_batch_verify_mixed(X):
    items, want = [], []
    for i in range(6):
        kws = synthetic.burn_inputs(40 + i)
        proof = _oracle_proof(kws, 64)
        air = _statement(X, kws)
        if i % 3 == 1:
            proof = _flip(proof, len(proof) // 2)
        if i % 3 == 2:
            air = (air[0], air[1], air[2] ^ 4)
        items.append((proof, air))
        want.append(i % 3 == 0)
    v = X.XfgBurnMintVerifier()
    assert v.batch_verify(items) == want
    assert v.batch_verify(items, threads=1) == want
    assert not v.verify_all(items) and v.verify_all([items[0], items[3]])
