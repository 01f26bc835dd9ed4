#!/bin/bash
# GPU box: kernel durations (rocprofv3 --kernel-trace --stats) of the configs[4] trace-LDE launch set
# for the current build and the ablation builds of scripts/abl_build.sh (XFG_LIB=ab/lib_<v>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for v in ${ABL_VARIANTS:-base nomath nostore}; do
  OUT=gpurun_out/abl_$v
  rm -rf $OUT && mkdir -p $OUT
  lib=""; [ $v != base ] && lib="XFG_LIB=$PWD/ab/lib_$v.so"
  env $lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/lde_c5.py 1 > $OUT/kt.log 2>&1 || { echo "$v failed"; tail -5 $OUT/kt.log; exit 1; }
  echo "== $v $(grep ' ms' $OUT/kt.log)"
  python3 scripts/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 4
done
