"""Host phases of single units (XFG_TRACE=1, stderr): one call of `count` proofs of 2^16 x 8 at a time,
after a warm call, so each unit runs alone as the window's last unit does -- where its serial tail
(sync, transcript replay, query planning, openings, serialisation) spends its time."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)
import synthetic
import xfgstark
pr = xfgstark.XfgBurnMintProver()
for count in (1, 16, 32):
    kws = [synthetic.burn_inputs(i) for i in range(count)]
    pr.prove_batch(kws, trace_length=1 << 16)
    print(f"--- {count} proofs", file=sys.stderr, flush=True)
    for _ in range(3):
        pr.prove_batch(kws, trace_length=1 << 16)
