"""Summarise a bench window's kernel trace (scripts/window_trace.sh): the timed window is the segment
with the most kernels between idle gaps > 0.5 ms (the warmup drains before the barrier); per 2 ms
bucket, the fraction of time any kernel runs and the mean number of kernels in flight."""
import csv
import os
import glob
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
ev.sort()
# segments separated by idle gaps > 0.5 ms; the timed window is the longest one
segs, cur, end = [], [ev[0]], ev[0][1]
for x in ev[1:]:
    if x[0] - end > 500_000:
        segs.append(cur)
        cur = []
    cur.append(x)
    end = max(end, x[1])
segs.append(cur)
for sg in segs:
    print(f"segment {(sg[0][0] - ev[0][0]) / 1e6:9.2f} ms: {len(sg):6d} kernels over "
          f"{(max(e for _, e, _ in sg) - sg[0][0]) / 1e6:8.2f} ms")
win = max(segs, key=len)
t0, t1 = win[0][0], max(e for _, e, _ in win)
print(f"window {len(win)} kernels, {(t1 - t0) / 1e6:.2f} ms from first start to last end")
B = 2_000_000
nb = (t1 - t0 + B - 1) // B
busy = [0] * nb
conc = [0] * nb
bounds = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
cur, last = 0, t0
for t, dlt in bounds:
    # account [last, t) with `cur` kernels in flight
    a = last
    while a < t:
        b = min(t, t0 + ((a - t0) // B + 1) * B)
        i = min((a - t0) // B, nb - 1)
        if cur > 0:
            busy[i] += b - a
        conc[i] += cur * (b - a)
        a = b
    cur += dlt
    last = t
print("bucket_ms  busy%  mean_kernels_in_flight")
for i in range(nb):
    span = min(B, t1 - (t0 + i * B))
    print(f"{i * 2:5d}-{i * 2 + 2:<4d} {100 * busy[i] / span:6.1f} {conc[i] / span:6.2f}")
tot_busy = sum(busy) / (t1 - t0)
print(f"whole window: busy {100 * tot_busy:.1f} %, mean in flight {sum(conc) / (t1 - t0):.2f}")

# the host's window (bench.py XFG_BENCH_TIMELINE: "window ns: start end", CLOCK_MONOTONIC like the trace)
import re
logs = glob.glob(d + "/log")
m = re.search(r"window ns: (\d+) (\d+)", open(logs[0]).read()) if logs else None
if m:
    h0, h1 = int(m.group(1)), int(m.group(2))
    print(f"host window {(h1 - h0) / 1e6:.2f} ms: first kernel {(t0 - h0) / 1e6:+.2f} ms after its start, "
          f"last kernel end {(h1 - t1) / 1e6:.2f} ms before its end")
    tail = sorted(win, key=lambda x: x[1])[-int(os.environ.get("TAIL", "12")):]
    for s_, e_, n_ in tail:
        print(f"  {(s_ - h0) / 1e6:8.2f} {(e_ - h0) / 1e6:8.2f}  {n_[:80]}")
