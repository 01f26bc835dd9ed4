"""Experiment (round 6): the 2^16 x 8 forward LDE for small launch sets (1-64 polynomials: one proof's
trace is 7, its composition / DEEP columns 1 each), all-coset pass A (ntt_pass_a_cos2 + ntt_pass_b_tq)
against one block per (tile, poly, coset) (ntt_pass_a + ntt_pass_b) -- the grid of the all-coset
pass A is 16 blocks per polynomial, so a single proof's launch sets under-fill the 256 CUs. Needs a
library built with -DXFG_EXP_SMALL (XFG_EXP_SMALL = smallest all-coset grid, XFG_EXP_NPOLY = polys per
set); run with XFG_LIB pointing at it."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark
pr = xfgstark.XfgBurnMintProver()
for np_ in (1, 2, 7, 14, 16, 28, 32, 64, 112, 224):
    os.environ["XFG_EXP_NPOLY"] = str(np_)
    row = []
    for route, small in (("cos2", "0"), ("percoset", "1000000")):
        os.environ["XFG_EXP_SMALL"] = small
        row.append((route, pr.bench_lde(1, 1 << 16, 8, 200)))
    print(np_, row, flush=True)
