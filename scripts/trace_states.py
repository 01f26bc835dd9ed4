"""Time split of a rocprofv3 kernel trace window into idle / a large grid running / only small grids
running (>= `big` workgroups counts as large), with the small-only time attributed per kernel.
usage: python3 scripts/trace_states.py <trace dir> <t0 ms> <t1 ms> [big]"""
import collections, csv, glob, sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
big_min = int(sys.argv[4]) if len(sys.argv) > 4 else 1024


def blocks(r):
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    w = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
    return g // max(1, w)


iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50], blocks(r)) for r in rows)
T0 = iv[0][0]
lo, hi = T0 + float(sys.argv[2]) * 1e6, T0 + float(sys.argv[3]) * 1e6
ev = []
for s, e, k, b in iv:
    s, e = max(s, lo), min(e, hi)
    if e > s:
        ev += [(s, 1, b >= big_min, k), (e, -1, b >= big_min, k)]
ev.sort(key=lambda x: (x[0], x[1]))
nb = ns = 0
t0 = lo
acc, small, active = collections.Counter(), collections.Counter(), collections.Counter()
for t, d, big, k in ev:
    dt = t - t0
    state = "idle" if nb + ns == 0 else "large" if nb > 0 else "small_only"
    acc[state] += dt
    if state == "small_only":
        live = [kk for kk, c in active.items() if c > 0]
        for kk in live:
            small[kk] += dt / len(live)
    if big:
        nb += d
    else:
        ns += d
    active[k] += d
    t0 = t
acc["idle"] += hi - t0 if t0 < hi else 0
tot = hi - lo
print(f"window {tot / 1e6:.1f} ms: " + ", ".join(f"{k} {100 * v / tot:.1f}%" for k, v in acc.items()))
for k, v in small.most_common(12):
    print(f"  small-only {v / 1e6:6.2f} ms  {k}")
