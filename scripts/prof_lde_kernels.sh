#!/bin/bash
# GPU box: rocprofv3 kernel stats of the trace-LDE launch sets (64 proofs) for each env setting in AB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/proflde
rm -rf $OUT && mkdir -p $OUT
i=0
for kv in $AB; do
  i=$((i+1))
  (cd /tmp && env ${kv//,/ } timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$i -o k -- python3 $OLDPWD/scripts/lde_only.py 64) > $OUT/k$i.log 2>&1 || { echo "prof $kv failed"; tail -5 $OUT/k$i.log; exit 1; }
  echo "== $kv"
  python3 - $OUT/k$i <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "ntt" in r["Name"]:
        print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
done
