"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals over a window of the
trace (default: the middle 60 % of the span of the named kernel's launches)"""
import csv, glob, sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
key = sys.argv[2] if len(sys.argv) > 2 else "ntt_pass_a_cos<8>"
rows = list(csv.DictReader(open(f)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [s for s, e, k in iv if key in k]
lo, hi = marks[len(marks) // 5], marks[4 * len(marks) // 5]
busy, cur_s, cur_e = 0, None, None
for s, e, k in iv:
    s, e = max(s, lo), min(e, hi)
    if e <= s:
        continue
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
span = hi - lo
print(f"window {span/1e6:.2f} ms, GPU busy (union of kernels) {busy/1e6:.2f} ms = {100*busy/span:.1f} %")
# idle gaps histogram
gaps, cur_e = [], None
for s, e, k in iv:
    if s < lo or s > hi:
        continue
    if cur_e is not None and s > cur_e:
        gaps.append(s - cur_e)
    cur_e = e if cur_e is None else max(cur_e, e)
gaps.sort(reverse=True)
print("largest idle gaps (us):", [round(g / 1e3, 1) for g in gaps[:15]], "count", len(gaps), "sum", round(sum(gaps) / 1e6, 2), "ms")
