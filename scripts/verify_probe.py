"""Batch verification of `count` configs[2] proofs (n = 2^16, beta 8): proofs/s through the GPU batch
verifier and the host verifier (16 threads), best of `reps`; with XFG_TRACE=1 the GPU path prints its
host phase times. usage: python3 scripts/verify_probe.py [count] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = 1 << 16
pr = xfgstark.XfgBurnMintProver()
kws = [synthetic.burn_inputs(i) for i in range(count)]
proofs = [p.to_bytes() for p in pr.prove_batch(kws, trace_length=n)]
items = [(p, xfgstark.air_consts(**kw)) for p, kw in zip(proofs, kws)]
v = xfgstark.XfgBurnMintVerifier()
for name, kw in (("gpu", {"gpu": pr}), ("host", {"threads": 16})):
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        ok = v.batch_verify(items, **kw)
        dt = time.perf_counter() - t
        assert all(ok)
        best = dt if best is None else min(best, dt)
    print(f"{name}: {count / best:.0f} proofs/s ({best * 1e3:.2f} ms per {count})", flush=True)
pr.close()
