#!/bin/bash
# GPU box: instruction-cache counters per kernel of one 64-proof batch (timing mode, scripts/stage_kernels.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/icache
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -oiE "SQC?_[A-Z_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST)[A-Z_]*" $OUT/counters.txt | sort -u | head -40
i=0
for grp in "$@"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 $OLDPWD/scripts/stage_kernels.py) > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; continue; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if any(s in k for s in ("leaves", "ntt", "fri", "tree", "constraint", "ood", "deep")):
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
