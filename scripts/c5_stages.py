"""configs[4] per-stage GPU times of one batch in timing mode (the batch is one unit on one stream, so
every kernel runs alone): 2^20-step trace, blowup 16, quadratic extension, 24 queries, grinding 4,
`count` proofs (default 4, bench.py config5's unit). usage: python3 scripts/c5_stages.py [count]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = 1 << 20
o = xfgstark.ProofOptions.reference()
o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
pr = xfgstark.XfgBurnMintProver(proof_options=o)
pr.prepare(count, n)
kws = [synthetic.burn_inputs(70_000 + i) for i in range(count)]
pr.set_timing(True)
for rep in range(2):
    pr.prove_batch(kws, trace_length=n)
    st = {k: round(v, 3) for k, v in pr.stage_times().items()}
print(json.dumps({"proofs": count, "stage_ms": st}))
pr.close()
