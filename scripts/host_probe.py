"""Where the host time of bench.py's pipelined loop goes: per step, the Python submit (marshalling
+ enqueue), the wait inside pending.result() and the to_bytes() copies; plus the box's CPU."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)
import xfgstark  # noqa: E402
import synthetic  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
per, n = 64, 1 << 16
pr = xfgstark.XfgBurnMintProver()
pr.prepare(per, n)
batches = [[synthetic.burn_inputs(k * per + i) for i in range(per)] for k in range(steps + 3)]
tsub = twait = tbytes = 0.0
pending = []


def collect(p):
    global twait, tbytes
    t = time.perf_counter()
    res = p.result()
    t2 = time.perf_counter()
    out = [r.to_bytes() for r in res]
    twait += t2 - t
    tbytes += time.perf_counter() - t2
    return out


for k, b in enumerate(batches):
    if k == 3:
        t0 = time.perf_counter()
        tsub = twait = tbytes = 0.0
    t = time.perf_counter()
    pending.append(pr.submit_batch(b, trace_length=n))
    tsub += time.perf_counter() - t
    if len(pending) >= depth:
        collect(pending.pop(0))
while pending:
    collect(pending.pop(0))
el = time.perf_counter() - t0
print(f"depth {depth}: {steps * per / el:.0f} proofs/s, per step: submit {1e3 * tsub / steps:.2f} ms, "
      f"wait {1e3 * twait / steps:.2f} ms, to_bytes {1e3 * tbytes / steps:.2f} ms, total {1e3 * el / steps:.2f} ms")
try:
    model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
except Exception:
    model = "?"
print(f"cpu: {model}, os.cpu_count {os.cpu_count()}, sched_getaffinity {len(os.sched_getaffinity(0))}, "
      f"loadavg {open('/proc/loadavg').read().split()[:3]}")
pr.close()
