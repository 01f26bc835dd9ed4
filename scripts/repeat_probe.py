"""Determinism probe: prove the same configs[4] input (n = 2^20, blowup 16, quadratic, 24 queries)
REPS times through one prover, synchronously, and report each proof's SHA-256 against the committed
oracle digest (tests/golden/config_proofs.json) with the first differing byte against proof 1.
usage: python3 scripts/repeat_probe.py [REPS]   (XFG_LIB selects the build; PREPARE=1 calls prepare(1, 2^20)
first, so that every lane's workspace exists before the first proof)"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    import synthetic
    import xfgstark
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    gold = json.load(open(os.path.join(ROOT, "tests/golden/config_proofs.json")))["config5"]
    o = xfgstark.ProofOptions.reference()
    o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
    pr = xfgstark.XfgBurnMintProver()
    pr._options = o
    kw = synthetic.burn_inputs(gold["source"])
    if os.environ.get("PREPARE"):
        pr.prepare(1, 1 << 20)
    first = None
    for r in range(reps):
        p = pr.prove_burn_mint(**kw, trace_length=1 << 20).to_bytes()
        sha = hashlib.sha256(p).hexdigest()
        diff = None
        if first is not None and p != first:
            diff = next(i for i in range(min(len(p), len(first))) if p[i] != first[i])
        first = first or p
        print(f"rep {r} done", file=sys.stderr, flush=True)
        print(f"rep {r}: len {len(p)} golden {sha == gold['sha256']} first_diff_vs_rep0 {diff}", flush=True)
    pr.close()


if __name__ == "__main__":
    main()
