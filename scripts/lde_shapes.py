"""Trace-LDE launch-set time (HIP events on the prover stream) for the four-step shapes the
radix-32 passes touch; env knobs (XFG_NTT_E, XFG_NTT_LTA, XFG_NTT_LTB) select the variant.
usage: python3 scripts/lde_shapes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark  # noqa: E402

pr = xfgstark.XfgBurnMintProver()
tag = " ".join(f"{k}={os.environ[k]}" for k in ("XFG_NTT_E", "XFG_NTT_LTA", "XFG_NTT_LTB") if k in os.environ)
for count, logn, beta in [(64, 16, 8), (16, 18, 4), (8, 19, 4), (4, 20, 16)]:
    ms = pr.bench_lde(count, 1 << logn, beta, 10)
    n = 1 << logn
    B = 8 * 7 * (n + n * beta) * count
    print(f"[{tag}] LDE count={count} n=2^{logn} beta={beta}: {ms:.3f} ms  {B / ms / 1e6:.1f} GB/s")
