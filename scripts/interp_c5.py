"""configs[4]-size interpolations alone (for rocprofv3 --kernel-trace): the trace's 28 columns of 2^20
(4 proofs x 7) and the composition's 8 columns of 2^21 (4 proofs x 2 extension coordinates), through
xfg_debug_interpolate (host copies around each call; the kernel trace isolates the passes)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark  # noqa: E402

pr = xfgstark.XfgBurnMintProver()
rng = np.random.default_rng(1)
P = (1 << 64) - (1 << 32) + 1
for npoly, logn in ((28, 20), (8, 21)):
    e = rng.integers(0, P, size=(npoly, 1 << logn), dtype=np.uint64)
    for _ in range(3):
        pr.debug_interpolate(e, 1 << logn)
    print(f"interpolated {npoly} x 2^{logn}", flush=True)
