"""Prove B pipelined 64-proof batches (n = 2^16, beta 8, the reference options) as bench.py does, for
a PMC pass: scripts/valu_ledger.sh runs it with B = 1 and B = 3 and takes the difference, so the
per-proof count excludes the setup kernels (tables, workspace warm-up)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

B = int(sys.argv[1])
per, n = 64, 1 << 16
pr = xfgstark.XfgBurnMintProver()
pr.prepare(per, n)
pend = [pr.submit_batch([synthetic.burn_inputs(k * per + i) for i in range(per)], trace_length=n) for k in range(B)]
for p in pend:
    assert all(not isinstance(r, Exception) for r in p.result())
pr.close()
print("batches", B)
