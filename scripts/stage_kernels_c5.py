"""One 4-proof configs[4] call (n = 2^20, blowup 16, quadratic extension, 24 queries, grinding 4) in
timing mode, 2 calls after a warm one: every kernel runs alone on the GPU. Run under rocprofv3
--kernel-trace for isolated per-kernel durations (scripts/kt_ab.sh STAGE_SCRIPT=...)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

per, n = 4, 1 << 20
pr = xfgstark.XfgBurnMintProver()
o = xfgstark.ProofOptions.reference()
o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
pr._options = o
pr.prepare(per, n)
pr.set_timing(True)
for k in range(3):
    pr.prove_batch([synthetic.burn_inputs(k * per + i) for i in range(per)], trace_length=n)
print({k: round(v, 3) for k, v in pr.stage_times().items()})
pr.close()
