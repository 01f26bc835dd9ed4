import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark, synthetic
pr = xfgstark.XfgBurnMintProver()
o = xfgstark.ProofOptions.reference()
o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
pr._options = o
n = 1 << 20
k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
kws = [synthetic.burn_inputs(7000 + i) for i in range(k)]
for r in range(3):
    t = time.perf_counter()
    pr.prove_batch(kws, trace_length=n)
    print(f"call {r}: {(time.perf_counter()-t)*1e3:.1f} ms", flush=True)
