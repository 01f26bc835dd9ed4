"""Completion times of the bench's pipelined steps (20 steps, depth 6, 64 proofs each): when each
batch was submitted and when its proofs were back, relative to the start of the timed region --
where the fill and drain of the pipeline go. usage: python3 scripts/pipe_timeline.py [steps] [depth]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n, per = 1 << 16, 64
pr = xfgstark.XfgBurnMintProver()
pr.prepare(per, n, buffers=int(os.environ.get('BUFS', depth)))
batches = [[synthetic.burn_inputs(k * per + i) for i in range(per)] for k in range(steps + 3)]
for rep in range(2):
    pend, log = [], []
    t0 = time.perf_counter()
    for i, b in enumerate(batches[:steps] if rep else batches[steps:]):
        ts = time.perf_counter() - t0
        pend.append((i, ts, pr.submit_batch(b, trace_length=n)))
        tq = time.perf_counter() - t0
        if len(pend) >= depth:
            j, s, p = pend.pop(0)
            r = p.result()
            log.append((j, s, tq, time.perf_counter() - t0))
    while pend:
        j, s, p = pend.pop(0)
        r = p.result()
        log.append((j, s, s, time.perf_counter() - t0))
    el = time.perf_counter() - t0
    if rep:
        for j, s, q, d in log:
            print(f"batch {j:3d} submit {s * 1e3:7.2f} ms (returned {q * 1e3:7.2f})  done {d * 1e3:7.2f} ms")
        print(f"total {el * 1e3:.2f} ms for {steps} steps = {el * 1e3 / steps:.3f} ms/step")
        gaps = [log[k][3] - log[k - 1][3] for k in range(1, len(log))]
        print("completion gaps ms:", " ".join(f"{g * 1e3:.2f}" for g in gaps))
pr.close()
