"""Deterministic synthetic burn inputs: SplitMix64 seeded per proof index.

burn = mint = 8,000,000 (0.8 XFG; 800 XFG is excluded because the reference truncates amounts
`as u32`, src/burn_mint_prover.rs:91, which breaks transition constraint r0), random 32-byte
tx prefix hash with a non-zero legacy u64, 20-byte recipient, 32-byte secret, network_id 1
(CLI fallback), target chain 42161, commitment version 1. Shared by tests/ and bench.py.
"""
SEED = 0x46472D535441524B  # "FG-STARK"
MASK = (1 << 64) - 1


def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & MASK
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return state, z ^ (z >> 31)


def _bytes(state, k):
    out = bytearray()
    while len(out) < k:
        state, v = splitmix64(state)
        out += v.to_bytes(8, "little")
    return state, bytes(out[:k])


def burn_inputs(index, seed=SEED):
    st = (seed ^ (index * 0xD1B54A32D192ED03)) & MASK
    st, tx = _bytes(st, 32)
    if int.from_bytes(tx[:8], "little") == 0:
        tx = b"\x01" + tx[1:]
    st, rcpt = _bytes(st, 20)
    st, secret = _bytes(st, 32)
    return dict(burn_amount=8_000_000, mint_amount=8_000_000, tx_prefix_hash=tx, recipient_address=rcpt,
                secret=secret, network_id=1, target_chain_id=42161, commitment_version=1)


# tests/test_data_package.json of the reference, marshalled as its CLI does
# (src/bin/xfg-stark-cli.rs:487-517: secret string zero-padded to 32 bytes, network_id "fuego-mainnet" -> 1)
REFERENCE_PACKAGE = dict(
    burn_amount=8_000_000, mint_amount=8_000_000,
    tx_prefix_hash=bytes.fromhex("7D0725F8E03021B99560ADD456C596FEA7D8DF23529E23765E56923B73236E4D"),
    recipient_address=bytes.fromhex("742d35Cc6634C0532925a3b8D4C9db96C4b4d8b6"),
    secret=b"dummy_secret_key".ljust(32, b"\0"), network_id=1, target_chain_id=42161, commitment_version=1)
