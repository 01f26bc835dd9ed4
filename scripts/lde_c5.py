"""C5-size trace LDE launch sets only (for profiling): 7 columns, n = 2^20, blowup 16"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark
pr = xfgstark.XfgBurnMintProver()
print(f"{pr.bench_lde(int(sys.argv[1]) if len(sys.argv) > 1 else 1, 1 << 20, 16, 5):.3f} ms")
