"""trace-LDE launch-set time for one split of n = R * C (XFG_NTT_LOGC) at several sizes"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark
pr = xfgstark.XfgBurnMintProver()
for logn, beta, cnt in ((16, 8, 64), (18, 8, 8), (20, 16, 1)):
    n = 1 << logn
    ms = pr.bench_lde(cnt, n, beta, 5)
    print(f"logC={os.environ.get('XFG_NTT_LOGC','auto')} n=2^{logn} beta={beta} x{cnt}: {ms:.3f} ms "
          f"{8*7*(n+beta*n)*cnt/ms/1e6:.0f} GB/s")
