"""Per-kernel time for ONE proving batch from a single-lane kernel trace: excludes the
xfg_bench_lde launches (grid.y = 7*64*... large) by taking the dispatches between the first
trace_gen_kernel of the last timed step and the next one."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
tg = [i for i, e in enumerate(ev) if "trace_gen_kernel" in e[2]]
# batches start at each trace_gen; use the second-to-last full batch (steady state)
if len(tg) < 3:
    print("not enough batches", len(tg)); sys.exit(0)
a, b = tg[-3], tg[-2]
win = ev[a:b]
span = win[-1][1] - win[0][0]
tot = defaultdict(float); cnt = defaultdict(int)
for s, e, n in win:
    tot[n] += e - s; cnt[n] += 1
busy = sum(tot.values())
print(f"batch span {span/1e6:.3f} ms, kernel time {busy/1e6:.3f} ms ({100*busy/span:.0f}% busy)")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k[:66]:66s} x{cnt[k]:3d} {v/1e6:8.3f} ms")
