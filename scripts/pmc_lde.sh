#!/bin/bash
# GPU box: PMC counter groups (one rocprofv3 --pmc pass each, arguments) on the trace-LDE launch sets
# alone -- SHAPE=c5 (one proof at 2^20 x 16, scripts/lde_c5.py 1) or c2 (64 proofs at 2^16 x 8) -- mean
# per kernel; `rocprofv3 -L` saved to gpurun_out/pmcl/counters.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcl
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
if [ "${SHAPE:-c5}" = c5 ]; then PROG="scripts/lde_c5.py 1"; else PROG="scripts/lde_only.py 64"; fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 $PROG > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if "ntt_pass" in k:
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")
PY
