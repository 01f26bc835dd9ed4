"""Data packages in, proof packages out: the host steps either side of the proving path.

Mirrors the reference's JSON schema (src/proof_data_schema.rs:11-67, 223-344) and the CLI
`generate` command (src/bin/xfg-stark-cli.rs:438-558, helpers hex_to_bytes / hex_to_u64 :715-736):

  StarkProofDataPackage (JSON) --validate / marshal--> prove_burn_mint kwargs
      --XfgBurnMintProver (MI355X)--> StarkProof --> proof package JSON
      {proof_data: [u8...], public_inputs: {...}, metadata: {...}}

Marshalling follows the CLI exactly, including its quirks: the secret is the UTF-8 bytes of
`secret_key` (not hex), zero padded / truncated to 32 bytes; the transaction hash and recipient
are hex-decoded then padded / truncated to 32 / 20 bytes; `network_id` is parsed as u32 with
fallback 1 ("fuego-mainnet" -> 1); target chain 42161 and commitment version 1 are fixed.
"""
import datetime
import json
import math
import re
from decimal import Decimal

VALID_BURN_XFG = (0.8, 800.0)
TARGET_CHAIN_ID = 42161  # Arbitrum One (xfg-stark-cli.rs generate)
COMMITMENT_VERSION = 1

_RUST_F64 = re.compile(r"^[+-]?((inf|infinity|nan)|(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)$", re.IGNORECASE)
_RUST_U32 = re.compile(r"^\+?\d+$")


class PackageError(ValueError):
    """XfgStarkError::ParseError (data package / hex input)"""


def rust_parse_f64(s):
    """str::parse::<f64>() or None (no surrounding whitespace, no '_' -- unlike float())"""
    if not isinstance(s, str) or not _RUST_F64.match(s):
        return None
    return float(s)


def rust_f64_display(x):
    """`{}` of an f64 in Rust: integral values without '.0', no exponent notation"""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    if x == int(x):
        return str(int(x))
    return format(Decimal(repr(x)), "f")


def rust_parse_u32(s):
    if not _RUST_U32.match(s):
        return None
    v = int(s)
    return v if v < 2 ** 32 else None


def hex_to_bytes(h):
    """xfg-stark-cli.rs:715-723: strip 0x, then hex::decode (FromHexError messages)"""
    h = h[2:] if h.startswith("0x") else h
    if len(h) % 2:
        raise PackageError("Odd number of digits")
    for i, ch in enumerate(h):
        if ch not in "0123456789abcdefABCDEF":
            raise PackageError(f"Invalid character {ch!r} at position {i}")
    return bytes.fromhex(h)


def hex_to_u64(h):
    """xfg-stark-cli.rs:725-736: little-endian u64 of the first 8 decoded bytes"""
    b = hex_to_bytes(h)
    if len(b) < 8:
        raise PackageError("Hex string too short for u64")
    return int.from_bytes(b[:8], "little")


def hex_to_u64_checked(h):
    """hex_to_u64 with the CLI's wrapping of hex errors ("Invalid hex string: ...")"""
    try:
        b = hex_to_bytes(h)
    except PackageError as e:
        raise PackageError(f"Invalid hex string: {e}")
    if len(b) < 8:
        raise PackageError("Hex string too short for u64")
    return int.from_bytes(b[:8], "little")


def _fit(b, n):
    return bytes(b[:n]).ljust(n, b"\0")


class ValidationResult:
    def __init__(self, errors, warnings):
        self.is_valid = not errors
        self.errors = errors
        self.warnings = warnings

    def __repr__(self):
        return f"ValidationResult(is_valid={self.is_valid}, errors={self.errors}, warnings={self.warnings})"


class StarkProofDataPackage:
    """proof_data_schema.rs StarkProofDataPackage: metadata, burn_transaction, recipient, secret,
    additional_data (kept as the parsed JSON object)"""

    REQUIRED = {"metadata": ("version", "created_at", "description", "network"),
                "burn_transaction": ("transaction_hash", "burn_amount_xfg", "burn_amount_atomic", "block_height",
                                     "timestamp", "network_id"),
                "recipient": ("ethereum_address",),
                "secret": ("secret_key",)}

    def __init__(self, data):
        for sect, fields in self.REQUIRED.items():  # serde: missing fields are parse errors
            if not isinstance(data.get(sect), dict):
                raise PackageError(f"missing field `{sect}`")
            for f in fields:
                if f not in data[sect]:
                    raise PackageError(f"missing field `{f}`")
        ints = {("burn_transaction", "burn_amount_atomic"), ("burn_transaction", "block_height"),
                ("burn_transaction", "timestamp")}
        for sect, fields in self.REQUIRED.items():
            for f in fields:
                v = data[sect][f]
                ok = (isinstance(v, int) and not isinstance(v, bool) and 0 <= v < 2 ** 64) if (sect, f) in ints \
                    else isinstance(v, str)
                if not ok:
                    raise PackageError(f"invalid type for `{f}`")
        self.data = data
        self.metadata = data["metadata"]
        self.burn_transaction = data["burn_transaction"]
        self.recipient = data["recipient"]
        self.secret = data["secret"]
        self.additional_data = data.get("additional_data", {})

    @classmethod
    def from_json(cls, text):
        try:
            return cls(json.loads(text))
        except json.JSONDecodeError as e:
            raise PackageError(str(e))

    @classmethod
    def load_from_file(cls, path):
        with open(path) as f:
            return cls.from_json(f.read())

    def to_json(self):
        return json.dumps(self.data, indent=2, ensure_ascii=False)

    @staticmethod
    def xfg_to_atomic_units(xfg):
        return int(xfg * 10_000_000.0)

    def get_mint_amount_atomic(self):
        return self.burn_transaction["burn_amount_atomic"]

    def get_mint_amount_heat(self):
        return self.burn_transaction["burn_amount_atomic"] / 10_000_000.0

    def validate(self):
        """StarkProofDataPackage::validate (proof_data_schema.rs:269-316), same messages"""
        errors, warnings = [], []
        amt = rust_parse_f64(self.burn_transaction["burn_amount_xfg"])
        amt = 0.0 if amt is None else amt
        if amt not in VALID_BURN_XFG:
            errors.append(f"Burn amount must be exactly 0.8 XFG or 800.0 XFG, got {rust_f64_display(amt)}")
        if self.burn_transaction["transaction_hash"].startswith("0x"):
            errors.append("Fuego transaction hash should not start with 0x")
        addr = self.recipient["ethereum_address"]
        if not addr.startswith("0x") or len(addr.encode()) != 42:
            errors.append("Ethereum address must be 0x-prefixed 40-character hex")
        if len(self.secret["secret_key"].encode()) < 8:
            errors.append("Secret key must be at least 8 characters")
        if self.burn_transaction["block_height"] == 0:
            warnings.append("Block height is 0 - please verify this is correct")
        if self.burn_transaction["timestamp"] == 0:
            warnings.append("Timestamp is 0 - please verify this is correct")
        return ValidationResult(errors, warnings)

    def prove_kwargs(self):
        """the CLI's marshalling of a validated package into prove_burn_mint arguments"""
        bt = self.burn_transaction
        try:  # the CLI's txn_hash_u64 = hex_to_u64(...) check, with its error wrapping
            hex_to_u64_checked(bt["transaction_hash"])
        except PackageError as e:
            raise PackageError(f"Invalid transaction hash: {e}")
        tx = _fit(hex_to_bytes(bt["transaction_hash"]), 32)
        try:
            rcpt = _fit(hex_to_bytes(self.recipient["ethereum_address"]), 20)
        except PackageError as e:
            raise PackageError(f"Invalid recipient address: {e}")
        secret = _fit(self.secret["secret_key"].encode(), 32)
        nid = rust_parse_u32(bt["network_id"]) if isinstance(bt["network_id"], str) else None
        return dict(burn_amount=bt["burn_amount_atomic"], mint_amount=self.get_mint_amount_atomic(),
                    tx_prefix_hash=tx, recipient_address=rcpt, secret=secret,
                    network_id=1 if nid is None else nid, target_chain_id=TARGET_CHAIN_ID,
                    commitment_version=COMMITMENT_VERSION)


def proof_package(package, proof_bytes, created_at=None):
    """the `generate` command's output object (proof_data_schema.rs StarkProof, :45-67)"""
    bt = package.burn_transaction
    created_at = created_at or datetime.datetime.now(datetime.timezone.utc).isoformat()
    return {
        "proof_data": list(proof_bytes),
        "public_inputs": {"burn_amount": bt["burn_amount_atomic"], "mint_amount": package.get_mint_amount_atomic(),
                          "txn_hash": bt["transaction_hash"], "recipient_hash": package.recipient["ethereum_address"],
                          "state": 0},
        "metadata": {"version": "1.0.0", "created_at": created_at,
                     "description": f"STARK proof for {bt['burn_amount_xfg']} XFG burn",
                     "network": package.metadata["network"]},
    }


def dumps_proof_package(obj):
    """serde_json::to_string_pretty layout (2-space indent, one array element per line)"""
    return json.dumps(obj, indent=2, ensure_ascii=False)


def load_proof_package(path_or_text):
    """-> (proof bytes, public_inputs, metadata) from a `generate` output file or its text"""
    text = path_or_text
    if not path_or_text.lstrip().startswith("{"):
        with open(path_or_text) as f:
            text = f.read()
    d = json.loads(text)
    data = d["proof_data"]
    if not isinstance(data, list) or any((not isinstance(x, int)) or x < 0 or x > 255 for x in data):
        raise PackageError("proof_data must be an array of u8")
    return bytes(data), d["public_inputs"], d["metadata"]


def generate_proofs(prover, packages, trace_length=64, created_at=None):
    """`generate` over many packages as ONE MI355X batch (xfg_prove_batch): validation errors are
    reported per package like the CLI does, valid ones are proven together.
    Returns a list of (proof package dict | None, ValidationResult | Exception)."""
    out = [None] * len(packages)
    todo, kws = [], []
    for i, p in enumerate(packages):
        v = p.validate()
        if not v.is_valid:
            out[i] = (None, v)
            continue
        try:
            kws.append(p.prove_kwargs())
            todo.append((i, v))
        except PackageError as e:
            out[i] = (None, e)
    if kws:
        res = prover.prove_batch(kws, trace_length=trace_length)
        for (i, v), r in zip(todo, res):
            out[i] = (None, r) if isinstance(r, Exception) else (proof_package(packages[i], r.to_bytes(), created_at), v)
    return out


def generate_proof(prover, input_file, output_file, trace_length=64, created_at=None):
    """xfg-stark-cli `generate <package.json> <proof.json>` on the MI355X prover"""
    pkg = StarkProofDataPackage.load_from_file(input_file)
    (obj, v), = generate_proofs(prover, [pkg], trace_length, created_at)
    if obj is None:
        if isinstance(v, ValidationResult):
            raise PackageError("Data package validation failed: " + "; ".join(v.errors))
        raise v
    with open(output_file, "w") as f:
        f.write(dumps_proof_package(obj))
    return obj
