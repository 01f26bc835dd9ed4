#!/bin/bash
# GPU box: per-kernel times (rocprofv3 --kernel-trace --stats) and SQ_INSTS_VALU of the trace-LDE
# launch set under NTT knob variants. SHAPE="count n blowup"; VARIANTS="name:ENV=..;..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
read -r CNT N BL <<< "${SHAPE:-64 65536 8}"
V="${VARIANTS:-base:}"
PROG="import sys; sys.path.insert(0, '$PWD/xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); print(f'{p.bench_lde($CNT, $N, $BL, 5):.3f} ms')"
IFS=';' read -ra VS <<< "$V"
for v in "${VS[@]}"; do
  name="${v%%:*}"; envs="${v#*:}"
  OUT=$PWD/gpurun_out/ldekt_$name
  rm -rf $OUT && mkdir -p $OUT
  (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -c "$PROG") > $OUT/kt.log 2>&1 || { echo "$name failed"; tail -5 $OUT/kt.log; exit 1; }
  (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc -o pmc -- python3 -c "$PROG") > $OUT/pmc.log 2>&1 || { echo "$name pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
  echo "== $name $(grep ' ms' $OUT/kt.log)"
  python3 scripts/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 3
  python3 - "$OUT/pmc" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if "ntt_pass" in k:
        print("   ", k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(d.items())})
PY
done
