"""configs[4] side measurement (bench.config5) over windows of 12 / 24 / 48 calls of 4 proofs, 6 in
flight: does the 12-call window of the bench line under-read the steady state? (profiles/r05/INDEX.md)"""
import os
import sys

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402

sys.path.insert(0, os.path.join(os.getcwd(), "xfg-stark_amd"))
import xfgstark  # noqa: E402

pr = xfgstark.XfgBurnMintProver()
for calls in (12, 24, 48, 12):
    r = bench.config5(pr, 0, batch=4, calls=calls, depth=6)
    print(calls, r["proofs_per_s"], r["ms_per_proof"], flush=True)
pr.close()
