#!/bin/bash
# kernel stats of the bench steps alone (no config-5 side measurement, no CPU baseline) + GPU busy union
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/steps
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o st -- python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-config5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 scripts/busy_union.py $OUT/trace > $OUT/busy.txt 2>&1; head -3 $OUT/busy.txt
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py $f 25 > $OUT/kstats.txt 2>&1; cat $OUT/kstats.txt
