"""Mean isolated duration (us) per kernel of the 64-proof launches (grid y = 64 x columns) in each
variant's kernel traces under gpurun_out/kt_ab/<variant>.<round>/ (scripts/kt_ab.sh)."""
import collections, csv, glob, os, sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(glob.glob(os.path.join(out, "*.*"))):
    if not os.path.isdir(d):
        continue
    name = os.path.basename(d).rsplit(".", 1)[0]
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            gy = int(r["Grid_Size_Y"])
            if gy % 64 == 0 and gy >= 64:  # the timed 64-proof batch (prepare runs 32-proof units)
                k = r["Kernel_Name"].split("(")[0][:60]
                acc[k][name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
names = sorted({n for k in acc for n in acc[k]})
print("kernel".ljust(62) + "".join(n[:12].rjust(13) for n in names))
for k in sorted(acc, key=lambda k: -max(sum(v) / len(v) for v in acc[k].values())):
    print(k.ljust(62) + "".join((f"{sum(acc[k][n]) / len(acc[k][n]):10.1f}({len(acc[k][n])})" if acc[k][n] else "-").rjust(13) for n in names))
