"""Per-stage device times of one config-5 batch (n = 2^20, blowup 16, quadratic extension, 24 queries)
and of one config-2 batch, from the prover's timing mode (HIP events between the stages of one lane).
usage: python3 scripts/c5_stages.py [batch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
pr = xfgstark.XfgBurnMintProver()
for name, n, opts in (("config5", 1 << 20, dict(field_extension=2, blowup_factor=16, num_queries=24)),
                      ("config2", 1 << 16, {})):
    o = xfgstark.ProofOptions.reference()
    for a, v in opts.items():
        setattr(o, a, v)
    pr._options = o
    kws = [synthetic.burn_inputs(7000 + i) for i in range(k if name == "config5" else 16)]
    pr.prove_batch(kws, trace_length=n)
    pr.set_timing(True)
    t = time.perf_counter()
    pr.prove_batch(kws, trace_length=n)
    dt = time.perf_counter() - t
    st = pr.stage_times()
    pr.set_timing(False)
    dev = sum(v for s, v in st.items() if not s.startswith("host"))
    print(f"{name}: {len(kws)} proofs, {dt * 1e3:.1f} ms wall, device stages {dev:.2f} ms")
    for s, v in st.items():
        print(f"  {s:18s} {v:8.3f} ms")
