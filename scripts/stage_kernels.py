"""One 64-proof batch (n=2^16, beta 8) in timing mode: the whole batch is one unit on one stream, so
every kernel runs alone on the GPU. Run under rocprofv3 --kernel-trace to get isolated per-kernel
durations (scripts/stage_kernels.sh)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

per, n = 64, 1 << 16
pr = xfgstark.XfgBurnMintProver()
pr.prepare(per, n)
pr.set_timing(True)
for k in range(3):
    pr.prove_batch([synthetic.burn_inputs(k * per + i) for i in range(per)], trace_length=n)
print({k: round(v, 3) for k, v in pr.stage_times().items()})
pr.close()
