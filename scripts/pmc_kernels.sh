#!/bin/bash
# GPU box: VALUBusy / occupancy / VALU instruction counts of every prover kernel (two short bench
# steps), one rocprofv3 --pmc pass per counter group; summary per kernel name
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmck
rm -rf $OUT && mkdir -p $OUT
i=0
for grp in "VALUBusy" "OccupancyPercent" "SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 scripts/host_probe.py 3 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    rows.append((m.get("SQ_INSTS_VALU", 0) * len(d.get("SQ_INSTS_VALU", [])), k, m))
for tot, k, m in sorted(rows, reverse=True)[:20]:
    print(f"{k:48s} valu_insts_total={tot/1e6:9.1f}M busy={m.get('VALUBusy',0):5.1f} occ={m.get('OccupancyPercent',0):5.1f}")
PY
