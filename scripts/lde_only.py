"""LDE launch sets only (for PMC collection): 64 proofs x 7 columns, n=2^16, blowup 8."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark
pr = xfgstark.XfgBurnMintProver()
ms = pr.bench_lde(int(sys.argv[1]) if len(sys.argv) > 1 else 64, 1 << 16, 8, 3)
print(f"{ms:.3f} ms")
