"""ASan + UBSan run of the untrusted-input path (CPU, no GPU).

libxfgstark's proof parser and host verifier (xfg-stark_amd/csrc/verifier.cpp) take attacker-supplied
bytes, like the reference's XfgBurnMintVerifier -> winterfell::verify (src/burn_mint_verifier.rs:186-283).
`make -C xfg-stark_amd sanitize` builds them host-only with -fsanitize=address,undefined together with
the mutation driver tests/sanitize/fuzz_verify.cpp; here the driver runs on oracle proofs (base field
and quadratic extension): every truncation, byte mutations at every offset, field elements >= p at
every offset, trailing bytes. The untouched proof must verify, every mutant must be rejected, and the
sanitizers must report nothing (they abort the driver on the first finding)."""
import os
import struct
import subprocess

import pytest

import oracle_lib as O
import synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "xfg-stark_amd", "build", "asan", "fuzz_verify")


@pytest.fixture(scope="module")
def fuzz_bin():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "xfg-stark_amd"), "sanitize"], check=True)
    return BIN


@pytest.mark.parametrize("n,blowup,ext,queries,stride", [(64, 8, 1, 42, 1), (64, 8, 2, 42, 2), (256, 4, 1, 24, 5)])
def test_mutated_proofs_rejected_under_asan_ubsan(fuzz_bin, tmp_path, n, blowup, ext, queries, stride):
    kw = synthetic.burn_inputs(700 + n + ext)
    st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                kw["recipient_address"], kw["secret"])
    assert st == 0
    opts = O.options(blowup=blowup, field_extension=ext, num_queries=queries)
    st, proof = O.prove(air, n, opts)
    assert st == 0
    pf, af = tmp_path / "proof.bin", tmp_path / "air.bin"
    pf.write_bytes(proof)
    af.write_bytes(struct.pack("<14Q", *air.pub, air.nullifier, air.commitment))
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:abort_on_error=0:detect_leaks=1:exitcode=77",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=78")
    r = subprocess.run([fuzz_bin, str(pf), str(af), str(queries), str(blowup), "4", str(ext), "8", "31", str(stride)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.startswith("checked ") and r.stdout.rstrip().endswith("accepted 0")
