"""Data-package -> inputs marshalling and proof-package JSON.

Mirrors src/proof_data_schema.rs (StarkProofDataPackage::validate :269-316, StarkProof :45-67) and
the CLI `generate` command (src/bin/xfg-stark-cli.rs:438-558, hex helpers :715-736). The package
below carries the field values of the reference's tests/test_data_package.json (as also recorded
in SURVEY.md §8(c)); its marshalled form must equal synthetic.REFERENCE_PACKAGE, the inputs the
committed golden proofs were made from."""
import json
import os

import pytest

import synthetic

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _package(**over):
    d = {
        "metadata": {"version": "1.0.0", "created_at": "2025-08-30T05:52:29.344873+00:00",
                     "description": "STARK proof for 0.8 XFG burn", "network": "fuego-mainnet"},
        "burn_transaction": {"transaction_hash": "7D0725F8E03021B99560ADD456C596FEA7D8DF23529E23765E56923B73236E4D",
                             "burn_amount_xfg": "0.8", "burn_amount_atomic": 8000000, "block_height": 819809,
                             "timestamp": 1756532538, "network_id": "fuego-mainnet"},
        "recipient": {"ethereum_address": "0x742d35Cc6634C0532925a3b8D4C9db96C4b4d8b6", "ens_name": None,
                      "label": None},
        "secret": {"secret_key": "dummy_secret_key", "salt": None, "hint": None},
        "additional_data": {},
    }
    for path, v in over.items():
        sect, f = path.split(".")
        d[sect][f] = v
    return d


@pytest.fixture(scope="module")
def K():
    from xfgstark import package
    return package


def test_reference_package_marshals_to_reference_inputs(K):
    p = K.StarkProofDataPackage.from_json(json.dumps(_package()))
    v = p.validate()
    assert v.is_valid and v.errors == [] and v.warnings == []
    assert p.prove_kwargs() == synthetic.REFERENCE_PACKAGE
    assert p.get_mint_amount_atomic() == 8000000 and p.get_mint_amount_heat() == 0.8


def test_validation_messages(K):
    bad = K.StarkProofDataPackage(_package(**{
        "burn_transaction.burn_amount_xfg": "1.5", "burn_transaction.transaction_hash": "0xabcd",
        "recipient.ethereum_address": "742d35Cc", "secret.secret_key": "short",
        "burn_transaction.block_height": 0, "burn_transaction.timestamp": 0}))
    v = bad.validate()
    assert not v.is_valid
    assert v.errors == ["Burn amount must be exactly 0.8 XFG or 800.0 XFG, got 1.5",
                        "Fuego transaction hash should not start with 0x",
                        "Ethereum address must be 0x-prefixed 40-character hex",
                        "Secret key must be at least 8 characters"]
    assert v.warnings == ["Block height is 0 - please verify this is correct",
                          "Timestamp is 0 - please verify this is correct"]
    # Rust f64 parsing / display: unparsable -> 0, integral values print without ".0"
    assert K.StarkProofDataPackage(_package(**{"burn_transaction.burn_amount_xfg": " 0.8"})).validate().errors == [
        "Burn amount must be exactly 0.8 XFG or 800.0 XFG, got 0"]
    assert K.StarkProofDataPackage(_package(**{"burn_transaction.burn_amount_xfg": "8e2"})).validate().is_valid
    assert K.StarkProofDataPackage(_package(**{"burn_transaction.burn_amount_xfg": "80"})).validate().errors == [
        "Burn amount must be exactly 0.8 XFG or 800.0 XFG, got 80"]


def test_cli_marshalling_quirks(K):
    # short hashes / addresses are zero padded, the secret is the key's UTF-8 bytes, network id u32
    p = K.StarkProofDataPackage(_package(**{
        "burn_transaction.transaction_hash": "0102030405060708", "burn_transaction.network_id": "7",
        "recipient.ethereum_address": "0x" + "ab" * 20, "secret.secret_key": "k" * 40}))
    kw = p.prove_kwargs()
    assert kw["tx_prefix_hash"] == bytes(range(1, 9)) + bytes(24)
    assert kw["recipient_address"] == b"\xab" * 20
    assert kw["secret"] == b"k" * 32 and kw["network_id"] == 7
    assert (kw["target_chain_id"], kw["commitment_version"]) == (42161, 1)
    for tx, msg in (("01020304", "Invalid transaction hash: Hex string too short for u64"),
                    ("0102030", "Invalid transaction hash: Invalid hex string: Odd number of digits"),
                    ("01020304050607zz", "Invalid transaction hash: Invalid hex string: Invalid character 'z' at position 14")):
        with pytest.raises(K.PackageError, match=msg.replace("(", r"\(")):
            K.StarkProofDataPackage(_package(**{"burn_transaction.transaction_hash": tx})).prove_kwargs()
    with pytest.raises(K.PackageError, match="Invalid recipient address: Invalid character 'x' at position 0"):
        K.StarkProofDataPackage(_package(**{"recipient.ethereum_address": "0xx" + "1" * 39})).prove_kwargs()
    with pytest.raises(K.PackageError, match="missing field `secret_key`"):
        d = _package()
        del d["secret"]["secret_key"]
        K.StarkProofDataPackage(d)


def test_proof_package_json_roundtrip(K, tmp_path):
    import xfgstark
    case = [c for c in json.load(open(os.path.join(GOLD, "proofs.json"))) if c["name"] == "pkg_n64_b8"][0]
    proof = bytes.fromhex(case["proof_hex"])
    pkg = K.StarkProofDataPackage(_package())
    obj = K.proof_package(pkg, proof, created_at="2025-08-30T06:00:00+00:00")
    text = K.dumps_proof_package(obj)
    assert text.startswith('{\n  "proof_data": [\n    ')  # serde_json pretty layout
    assert obj["public_inputs"] == {"burn_amount": 8000000, "mint_amount": 8000000,
                                    "txn_hash": pkg.burn_transaction["transaction_hash"],
                                    "recipient_hash": "0x742d35Cc6634C0532925a3b8D4C9db96C4b4d8b6", "state": 0}
    assert obj["metadata"]["description"] == "STARK proof for 0.8 XFG burn"
    f = tmp_path / "proof.json"
    f.write_text(text)
    data, pub, meta = K.load_proof_package(str(f))
    assert data == proof and pub == obj["public_inputs"] and meta == obj["metadata"]
    p = xfgstark.StarkProof.from_bytes(data)
    assert p.trace_length == 64
    assert xfgstark.XfgBurnMintVerifier().verify_burn_mint(p, **pkg.prove_kwargs())
