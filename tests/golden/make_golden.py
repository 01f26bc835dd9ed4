"""Regenerates tests/golden/*.json from the CPU oracle (oracle/liboracle.so).

Hash KATs are published vectors (BLAKE3 spec test vectors, Keccak-256) plus the reference's own
KAT (src/lib.rs:135-161); they are typed in here as data and checked against the oracle, never
produced by it. Proof fixtures ARE produced by the oracle (parity unpinned against real
Winterfell: see oracle/oracle.h) and pin the restatement against regressions and the GPU path.
Usage: python tests/golden/make_golden.py            (hash KATs, reference KATs, proofs.json)
       python tests/golden/make_golden.py --configs  (config_proofs.json: the benchmark shapes, ~2 min
                                                      on 8 processes)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle_lib as O  # noqa: E402
import synthetic  # noqa: E402

KATS = {
    "blake3": [  # BLAKE3 official test vectors (input = bytes i % 251, hash mode, 32-byte output)
        {"input_hex": "", "digest": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"},
        {"input_hex": "00", "digest": "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213"},
        {"input_hex": "0001", "digest": "7b7015bb92cf0b318037702a6cdd81dee41224f734684c2c122cd6359cb1ee63"},
        {"input_hex": "616263", "digest": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"},
    ],
    "keccak256": [
        {"input_hex": "", "digest": "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"},
        {"input_hex": "616263", "digest": "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"},
        # reference src/lib.rs:141-149 (Fuego network id)
        {"input_hex": b"93385046440755750514194170694064996624".hex(),
         "digest": "6430829be74c2d9892a5122aa2f2daac3ee9850f086a8985941e7fb4bde60fcf"},
    ],
    # reference src/lib.rs:151-160: first 8 digest bytes LE mod (2^63 - 1)
    "network_id_field": {"digest_hex": "6430829be74c2d9892a5122aa2f2daac3ee9850f086a8985941e7fb4bde60fcf",
                         "mod": (1 << 63) - 1, "value": 1742133188492406885},
}


def reference_kats():
    """inputs + expected outputs from the reference's own tests / fixtures (values checked here)"""
    pkg = synthetic.REFERENCE_PACKAGE
    st, air = O.air_from_inputs(pkg["burn_amount"], pkg["mint_amount"], pkg["tx_prefix_hash"],
                                pkg["recipient_address"], pkg["secret"])
    assert st == 0
    return {
        # tests/test_data_package.json marshalled as src/bin/xfg-stark-cli.rs:487-517 does
        "test_data_package": {
            "inputs": {k: (v.hex() if isinstance(v, bytes) else v) for k, v in pkg.items()},
            "pub_inputs": list(air.pub), "secret_element": air.secret, "nullifier": air.nullifier,
            "commitment": air.commitment},
        # src/burn_mint_prover.rs:303-315
        "secret_conversion": {"secret_hex": "0102030405060708", "element": 0x04030201},
        # src/burn_mint_prover.rs:257-301 (status: 0 ok, 1 burn, 2 mint, 3 tx hash, 4 recipient)
        "validation": [
            {"burn": 8000000, "mint": 8000000, "tx_zero": False, "rlen": 20, "status": 0},
            {"burn": 0, "mint": 8000000, "tx_zero": False, "rlen": 20, "status": 1},
            {"burn": 8000000001, "mint": 8000000, "tx_zero": False, "rlen": 20, "status": 1},
            {"burn": 8000000, "mint": 0, "tx_zero": False, "rlen": 20, "status": 2},
            {"burn": 8000000, "mint": 16000000, "tx_zero": False, "rlen": 20, "status": 2},
            {"burn": 8000000, "mint": 8000000, "tx_zero": True, "rlen": 20, "status": 3},
            {"burn": 8000000, "mint": 8000000, "tx_zero": False, "rlen": 19, "status": 4},
            {"burn": 8000000000, "mint": 8000000000, "tx_zero": False, "rlen": 20, "status": 0},
        ],
        # src/burn_mint_air.rs:659-700 validate_state_transitions: d(d-1) == 0
        "state_transitions": [[0, 1, True], [1, 2, True], [2, 3, True], [1, 1, True], [0, 2, False],
                              [2, 0, False]],
    }


CASES = [  # (name, input source, n, blowup[, other ProofOptions])
    ("pkg_n64_b8", "package", 64, 8),
    ("pkg_n64_b4", "package", 64, 4),
    ("syn0_n1024_b4", 0, 1024, 4),   # config 1 shape (2^10 steps, blowup 4)
    ("syn1_n1024_b8", 1, 1024, 8),
    ("syn2_n4096_b8", 2, 4096, 8),
    ("syn0_n65536_b8", 0, 65536, 8),  # config 2 shape (2^16 steps, blowup 8)
    # FieldExtension::Quadratic (config 5's field): 16-byte E elements after the trace commitment
    ("pkg_n64_b8_quad", "package", 64, 8, {"field_extension": 2}),
    ("syn3_n4096_b16_quad_q24", 3, 4096, 16, {"field_extension": 2, "num_queries": 24}),
    ("syn4_n65536_b8_quad", 4, 65536, 8, {"field_extension": 2}),
]


def proof_fixtures():
    out = []
    for case in CASES:
        name, src, n, b = case[:4]
        extra = case[4] if len(case) > 4 else {}
        kw = synthetic.REFERENCE_PACKAGE if src == "package" else synthetic.burn_inputs(src)
        st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                    kw["recipient_address"], kw["secret"], kw["network_id"],
                                    kw["target_chain_id"], kw["commitment_version"])
        assert st == 0
        opts = O.options(blowup=b, **extra)
        st, proof = O.prove(air, n, opts)
        assert st == 0 and O.verify(air, proof, opts) == 0, name
        rec = {"name": name, "source": src, "n": n, "blowup": b, "len": len(proof),
               "sha256": hashlib.sha256(proof).hexdigest()}
        if extra:
            rec["options"] = extra
        if n <= 64:
            rec["proof_hex"] = proof.hex()
        out.append(rec)
        print(name, len(proof), rec["sha256"][:16])
    return out


# BASELINE configs[2]: the 128 proofs test_config2_full_batch_in_flight makes (two 64-proof batches,
# synthetic.burn_inputs(0..127), n = 2^16, blowup 8, reference options 42/8/4/None/8/31)
C2_N, C2_COUNT = 1 << 16, 128
# BASELINE configs[4] as bench.py's config5() and test_config5_quadratic_2p20_blowup16 run it:
# n = 2^20, blowup 16, quadratic extension, 24 queries, grinding 4, folding 8, remainder 31
C5_N, C5_SOURCE = 1 << 20, 5005
C5_OPTIONS = {"blowup": 16, "field_extension": 2, "num_queries": 24}
# bench.py config5()'s 4-proof batch (synthetic.burn_inputs(50000 + i)), for the pipelined configs[4] test
C5_BATCH_SOURCES = [50_000 + i for i in range(4)]


def _prove_digest(args):
    src, n, extra = args
    kw = synthetic.burn_inputs(src)
    st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                kw["recipient_address"], kw["secret"], kw["network_id"],
                                kw["target_chain_id"], kw["commitment_version"])
    assert st == 0
    opts = O.options(**extra)
    st, proof = O.prove(air, n, opts)
    assert st == 0 and O.verify(air, proof, opts) == 0, (src, n)
    return {"source": src, "len": len(proof), "sha256": hashlib.sha256(proof).hexdigest()}


def config_fixtures(procs=8):
    """digests of whole oracle proofs at the benchmark shapes (the oracle is single-threaded per
    proof, so the 128 configs[2] proofs run on a process pool)"""
    import multiprocessing as mp
    with mp.get_context("fork").Pool(procs) as pool:
        c5 = pool.apply_async(_prove_digest, ((C5_SOURCE, C5_N, C5_OPTIONS),))
        c5b = pool.map_async(_prove_digest, [(i, C5_N, C5_OPTIONS) for i in C5_BATCH_SOURCES], chunksize=1)
        c2 = pool.map(_prove_digest, [(i, C2_N, {}) for i in range(C2_COUNT)], chunksize=1)
        c5, c5b = c5.get(), c5b.get()
    print("config5", c5["len"], c5["sha256"][:16])
    c5opts = {k: v for k, v in C5_OPTIONS.items() if k != "blowup"}
    return {"config2_batch": {"n": C2_N, "blowup": 8, "options": {}, "proofs": c2},
            "config5": dict(c5, n=C5_N, blowup=16, options=c5opts),
            "config5_batch": {"n": C5_N, "blowup": 16, "options": c5opts, "proofs": c5b}}


def main():
    if "--configs" in sys.argv:
        with open(os.path.join(HERE, "config_proofs.json"), "w") as f:
            json.dump(config_fixtures(), f, indent=1)
        return
    for v in KATS["blake3"]:
        assert O.blake3(bytes.fromhex(v["input_hex"])).hex() == v["digest"], v
    for v in KATS["keccak256"]:
        assert O.keccak256(bytes.fromhex(v["input_hex"])).hex() == v["digest"], v
    with open(os.path.join(HERE, "kat_hashes.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(reference_kats(), f, indent=1)
    with open(os.path.join(HERE, "proofs.json"), "w") as f:
        json.dump(proof_fixtures(), f, indent=1)


if __name__ == "__main__":
    main()
