"""GPU busy analysis from a rocprofv3 kernel_trace.csv: union of kernel intervals, gaps, and
per-kernel exclusive-ish time within a window (the timed bench steps)."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_Y"])) for r in rows)
t0, t1 = ev[0][0], max(e[1] for e in ev)
# union
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, n, gy in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1-t0)/1e6:.2f} ms, busy {busy/1e6:.2f} ms ({100*busy/(t1-t0):.1f}%), gaps>50us: {sum(g for g in gaps if g>50000)/1e6:.2f} ms in {sum(1 for g in gaps if g>50000)}")
# attribute time slices to the set of running kernels (split equally among concurrent)
pts = sorted(set([s for s, *_ in ev] + [e for _, e, *_ in ev]))
share = defaultdict(float)
import bisect
active = []
starts = defaultdict(list)
for i, (s, e, n, gy) in enumerate(ev):
    starts[s].append(i)
ends = defaultdict(list)
for i, (s, e, n, gy) in enumerate(ev):
    ends[e].append(i)
act = set()
prev = None
for p in pts:
    if prev is not None and act:
        dt = p - prev
        for i in act:
            share[ev[i][2]] += dt / len(act)
    for i in ends.get(p, []):
        act.discard(i)
    for i in starts.get(p, []):
        act.add(i)
    prev = p
tot = sum(share.values())
for k, v in sorted(share.items(), key=lambda x: -x[1])[:22]:
    print(f"{k[:70]:70s} {v/1e6:8.2f} ms {100*v/tot:5.1f}%")
