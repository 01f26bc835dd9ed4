"""Trace-LDE launch sets of `count` proofs (xfg_bench_lde: pass A into scratch, pass B into the LDE,
buffers reused across iterations) for count = 1 .. 64: per-proof time and the HBM-roofline fraction
at the algorithmic 8 * 7 * (n + N) bytes per proof -- does a set whose intermediate fits the 256 MB
MALL run faster per proof?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark  # noqa: E402

pr = xfgstark.XfgBurnMintProver()
n, beta = 1 << 16, 8
pr.bench_lde(64, n, beta, 40)  # clocks up
for count in [int(x) for x in (sys.argv[1:] or "1 2 4 8 16 32 64".split())]:
    iters = max(20, 2560 // count)
    ms = pr.bench_lde(count, n, beta, iters)
    alg = 8 * 7 * (n + n * beta) * count
    print(f"count {count:3d}: {ms:8.3f} ms per set, {ms / count * 1e3:7.1f} us per proof, "
          f"{alg / (ms * 1e-3) / 1e12:5.2f} TB/s = {alg / (ms * 1e-3) / 8e12 * 100:5.1f} % of 8 TB/s "
          f"(scratch + LDE {2 * 8 * 7 * n * beta * count / 2**20:6.0f} MiB)", flush=True)
