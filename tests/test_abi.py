"""CPU-side checks of the product boundary: libxfgstark.so loads, exports every symbol the C header
declares, and its host logic (options, marshalling, validation errors) matches the reference
(src/burn_mint_prover.rs:27-41, 62-118, 132-221) and the oracle -- no GPU compute here."""
import ctypes as C
import os
import re

import pytest

import oracle_lib as O
import synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "xfg_stark.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xfg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import xfgstark
    lib = C.CDLL(xfgstark.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s


def test_library_is_gfx950_code_object():
    import subprocess
    import xfgstark
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", xfgstark.LIB_PATH], capture_output=True,
                         text=True).stdout if os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf") else ""
    if not out:
        pytest.skip("llvm-readelf unavailable")
    assert ".hip_fatbin" in out
    data = open(xfgstark.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_default_options_match_reference():
    import xfgstark
    o = xfgstark.ProofOptions.reference()
    assert (o.num_queries, o.blowup_factor, o.grinding_factor, o.field_extension, o.fri_folding_factor,
            o.fri_remainder_max_degree) == (42, 8, 4, 1, 8, 31)


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_marshalling_matches_oracle(idx):
    import xfgstark
    kw = synthetic.burn_inputs(idx)
    pub, nf, cm = xfgstark.air_consts(**kw)
    st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"], kw["recipient_address"],
                                kw["secret"], kw["network_id"], kw["target_chain_id"], kw["commitment_version"])
    assert st == 0
    assert pub == list(air.pub) and nf == air.nullifier and cm == air.commitment


def test_marshalling_reference_package():
    import xfgstark
    pub, nf, cm = xfgstark.air_consts(**synthetic.REFERENCE_PACKAGE)
    assert (pub[2], pub[3], nf, cm) == (4163176317, 4125078127, 2424340740, 44334705)


@pytest.mark.parametrize("burn,mint,tx0,rlen,slen,status", [
    (0, 8_000_000, 1, 20, 32, 1), (8_000_000_001, 8_000_000, 1, 20, 32, 1), (8_000_000, 0, 1, 20, 32, 2),
    (8_000_000, 16_000_000, 1, 20, 32, 2), (8_000_000, 8_000_000, 0, 20, 32, 3), (8_000_000, 8_000_000, 1, 19, 32, 4),
    (8_000_000, 8_000_000, 1, 20, 3, 5), (8_000_000, 8_000_000, 1, 20, 6, 5)])
def test_validation_errors(burn, mint, tx0, rlen, slen, status):
    import xfgstark
    tx = bytes([tx0]) + bytes(31)
    with pytest.raises(xfgstark.XfgStarkError) as e:
        xfgstark.air_consts(burn, mint, tx, b"\x12" * rlen, b"\x2a" * slen)
    assert e.value.status == status


def test_proof_size_bound_covers_oracle_sizes():
    import xfgstark
    lib = C.CDLL(xfgstark.LIB_PATH)
    lib.xfg_proof_size_bound.restype = C.c_size_t
    o = xfgstark.ProofOptions.reference()._c()
    import json
    for case in json.load(open(os.path.join(ROOT, "tests", "golden", "proofs.json"))):
        o.blowup_factor = case["blowup"]
        assert lib.xfg_proof_size_bound(C.c_uint64(case["n"]), C.byref(o)) >= case["len"]


@pytest.mark.parametrize("n,beta,q,ext,rem", [
    (8, 2, 15, 1, 1), (64, 4, 200, 1, 7), (64, 4, 255, 2, 7), (256, 8, 42, 1, 31), (256, 16, 128, 2, 3),
    (1024, 8, 42, 1, 31), (1024, 4, 100, 2, 255), (512, 2, 255, 1, 0)])
def test_proof_size_bound_is_tight_upper_bound(n, beta, q, ext, rem):
    """the bound a fixed-size exchange record is sized by (bench.Exchange): never below a real proof
    (the oracle's, same serialisation), including shapes where the queries fill the Merkle trees"""
    import xfgstark
    lib = C.CDLL(xfgstark.LIB_PATH)
    lib.xfg_proof_size_bound.restype = C.c_size_t
    o = xfgstark.ProofOptions(q, beta, 0, ext, 8, rem)._c()
    bound = lib.xfg_proof_size_bound(C.c_uint64(n), C.byref(o))
    opts = O.options(num_queries=q, blowup=beta, grinding=0, field_extension=ext, fri_rem_max_deg=rem)
    for i in range(3):
        kw = synthetic.burn_inputs(i)
        st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                    kw["recipient_address"], kw["secret"])
        st, proof = O.prove(air, n, opts)
        assert st == 0
        assert len(proof) <= bound, (len(proof), bound)


def test_proof_size_bound_configs2():
    """configs[2] (2^16, blowup 8, 42/8/4/None/8/31): golden proof ~78 KB, bound within 1.35x"""
    import json
    import xfgstark
    lib = C.CDLL(xfgstark.LIB_PATH)
    lib.xfg_proof_size_bound.restype = C.c_size_t
    o = xfgstark.ProofOptions.reference()._c()
    bound = lib.xfg_proof_size_bound(C.c_uint64(1 << 16), C.byref(o))
    lens = [c["len"] for c in json.load(open(os.path.join(ROOT, "tests", "golden", "proofs.json")))
            if c["n"] == 1 << 16 and c["blowup"] == 8 and "options" not in c]
    assert lens and all(ln <= bound < 1.35 * ln for ln in lens), (lens, bound)


def test_no_gpu_means_loud_failure():
    import torch
    import xfgstark
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(xfgstark.XfgStarkError):
        xfgstark.XfgBurnMintProver()


def test_host_field_arithmetic():
    import random
    import xfgstark
    lib = C.CDLL(xfgstark.LIB_PATH)
    P = 0xFFFFFFFF00000001
    out = (C.c_uint64 * 3)()
    rng = random.Random(5)
    edge = [0, 1, 2, P - 1, P - 2, 2**32 - 1, 2**32, 2**32 + 1, 2**63, P - 2**32]
    pairs = [(a, b) for a in edge for b in edge] + [(rng.randrange(P), rng.randrange(P)) for _ in range(3000)]
    for a, b in pairs:
        assert lib.xfg_selftest_field(C.c_uint64(a), C.c_uint64(b), out) == 0
        assert list(out) == [a * b % P, (a + b) % P, (a - b) % P], (a, b)
