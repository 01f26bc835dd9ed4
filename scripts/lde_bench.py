"""Time the trace-LDE launch set (HIP events on the prover stream) for a few shapes."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark
pr = xfgstark.XfgBurnMintProver()
for count, logn, beta in [(64, 16, 8), (8, 16, 8), (1, 16, 8), (4, 20, 16)]:
    ms = pr.bench_lde(count, 1 << logn, beta, 10)
    n = 1 << logn
    B = 8 * 7 * (n + n * beta) * count
    print(f"LDE count={count} n=2^{logn} beta={beta}: {ms:.3f} ms  {B/ms/1e6:.1f} GB/s  ({B/ms/1e6/8000*100:.1f}% of 8 TB/s)")
