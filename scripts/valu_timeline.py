"""VALU issue demand of the pipelined bench over time: each kernel's wave instructions (mean per
launch of that kernel name and grid, from the --pmc run) spread evenly over its duration in the
kernel trace; the sum over concurrent kernels per 50 us bucket against the chip's issue capacity
(1024 SIMDs x 2.38 GHz / 4.3 cycles per wave instruction, the measured half-rate ceiling)."""
import csv, glob, sys, collections
out = sys.argv[1]
tr = list(csv.DictReader(open(glob.glob(out + "/t/**/*kernel_trace.csv", recursive=True)[0])))
pm = list(csv.DictReader(open(glob.glob(out + "/p/**/*counter_collection.csv", recursive=True)[0])))
key = lambda name, grid: (name, grid)
acc = collections.defaultdict(list)
for r in pm:
    if r["Counter_Name"] == "SQ_INSTS_VALU":
        acc[key(r["Kernel_Name"], r["Grid_Size"])].append(float(r["Counter_Value"]))
per = {k: sum(v) / len(v) for k, v in acc.items()}
ev = []
for r in tr:
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    k = key(r["Kernel_Name"], str(g))
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], per.get(k)))
ev.sort()
missing = sum(1 for e in ev if e[3] is None)
# the pipelined steps: the longest run of kernels without a host-side gap of more than 1 ms (the
# synchronous batch, the LDE micro-benchmark and the stage-timing batch after it are separated by
# such gaps); its first quarter (warm-up steps) is skipped
runs, cs, ce, n = [], ev[0][0], ev[0][1], 0
for s_, e_, k_, w_ in ev:
    if s_ > ce + 1_000_000:
        runs.append((n, cs, ce)); cs, n = s_, 0
    ce, n = max(ce, e_), n + 1
runs.append((n, cs, ce))
n_, cs, ce = max(runs)
t0, t1 = cs + (ce - cs) // 4, ce
B = 50_000  # ns
nb = (t1 - t0) // B + 1
dem = [0.0] * nb
busy = [0] * nb
for s, e, k, w in ev:
    if e <= t0 or w is None:
        continue
    s2 = max(s, t0)
    rate = w / max(1, e - s)  # wave-instr per ns
    b = (s2 - t0) // B
    while b < nb and t0 + b * B < e:
        lo, hi = max(s2, t0 + b * B), min(e, t0 + (b + 1) * B)
        dem[b] += rate * (hi - lo)
        busy[b] = 1
        b += 1
cap = 1024 * 2.38 / 4.3 * B  # wave instructions per bucket at the ceiling
util = [d / cap for d in dem]
import statistics
print(f"window {(t1 - t0) / 1e6:.2f} ms, {nb} buckets of {B // 1000} us, kernels without a VALU count: {missing}")
print(f"mean VALU demand / ceiling {statistics.mean(util):.3f}; buckets with any kernel {sum(busy) / nb:.3f}")
hist = collections.Counter(min(9, int(u * 10)) for u in util)
print("demand histogram (tenths of the ceiling):", [hist.get(i, 0) for i in range(10)])
# what runs in low-demand buckets
low = collections.Counter()
for s, e, k, w in ev:
    if e <= t0:
        continue
    b0, b1 = max(0, (s - t0) // B), min(nb - 1, (e - t0) // B)
    for b in range(b0, b1 + 1):
        if util[b] < 0.5:
            low[k[:60]] += 1
print("kernels present in buckets below half the ceiling:", low.most_common(12))
# demand per bucket as one character (0-9 = tenths of the ceiling), 100 buckets (5 ms) per line
line = "".join(str(min(9, int(u * 10))) for u in util)
for i in range(0, len(line), 100):
    print(f"{i * B // 1000:6d} us  {line[i:i + 100]}")
