"""Batch verification throughput: host threads (xfg_verify_batch) vs GPU (xfg_verify_batch_gpu),
proofs of the bench workload (2^16 steps, blowup 8)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark, synthetic
pr = xfgstark.XfgBurnMintProver()
n, k = 1 << 16, int(sys.argv[1]) if len(sys.argv) > 1 else 512
kws = [synthetic.burn_inputs(i) for i in range(64)]
proofs = [p.to_bytes() for p in pr.prove_batch(kws, trace_length=n)]
airs = [xfgstark.air_consts(**kw) for kw in kws]
items = [(proofs[i % 64], airs[i % 64]) for i in range(k)]
v = xfgstark.XfgBurnMintVerifier()
for name, fn in (("host", lambda: v.batch_verify(items, threads=16)), ("gpu", lambda: v.batch_verify(items, gpu=pr))):
    assert all(fn())
    t = time.perf_counter()
    for _ in range(3):
        fn()
    dt = (time.perf_counter() - t) / 3
    print(f"{name}: {k} proofs in {dt*1e3:.1f} ms -> {k/dt:.0f} proofs/s")
if os.environ.get("XFG_TRACE") == "1":  # Python-side share of one GPU call
    import cProfile, pstats
    cProfile.run("v.batch_verify(items, gpu=pr)", "/tmp/vb.prof")
    pstats.Stats("/tmp/vb.prof").sort_stats("cumulative").print_stats(12)
