"""Config 5 timing: n = 2^20, blowup 16, quadratic extension, 24 queries (one proof per call)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark, synthetic
pr = xfgstark.XfgBurnMintProver()
o = xfgstark.ProofOptions.reference()
o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
pr._options = o
n = 1 << 20
for k in (1, 2, 4):
    kws = [synthetic.burn_inputs(7000 + i) for i in range(k)]
    pr.prove_batch(kws, trace_length=n)
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        pr.prove_batch(kws, trace_length=n)
    dt = (time.perf_counter() - t) / reps
    print(f"batch {k}: {dt*1e3:.1f} ms per call, {k/dt:.2f} proofs/s")
ms = pr.bench_lde(1, n, 16, 5)
print(f"trace LDE 7 cols 2^20 x16: {ms:.3f} ms, {8*7*(n + 16*n)/ms/1e6:.1f} GB/s algorithmic")
