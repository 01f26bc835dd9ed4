#!/bin/bash
# GPU box: kernel times and PMC (VALU busy / instructions / occupancy / HBM bytes) of the configs[4]
# trace LDE alone (2^20 steps, blowup 16, one proof = 7 polys), one rocprofv3 pass per counter group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/c5p
rm -rf $OUT && mkdir -p $OUT
PROG="import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); o = xfgstark.ProofOptions.reference(); o.field_extension, o.blowup_factor = 2, 16
p._options = o; p.prepare(1, 1 << 20); print('lde ms', p.bench_lde(1, 1 << 20, 16, 5))"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -c "$PROG" > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
cat $OUT/kt.log | grep "lde ms"
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); head -8 "$f"
i=0
for grp in "VALUBusy OccupancyPercent" "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 -c "$PROG" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
