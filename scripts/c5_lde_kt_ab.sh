#!/bin/bash
# GPU box: per-kernel times (rocprofv3 --kernel-trace --stats) of the configs[4] trace-LDE launch set
# of library builds: VARIANTS="name:XFG_LIB=ab/libX.so;..." (an empty setting = the in-tree build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
V="${VARIANTS:-base:}"
IFS=';' read -ra VS <<< "$V"
for v in "${VS[@]}"; do
  name="${v%%:*}"; envs="${v#*:}"
  OUT=gpurun_out/c5kt_$name
  rm -rf $OUT && mkdir -p $OUT
  env $envs timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/lde_c5.py 1 > $OUT/kt.log 2>&1 || { echo "$name failed"; tail -5 $OUT/kt.log; exit 1; }
  echo "== $name $(grep ' ms' $OUT/kt.log)"
  python3 scripts/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 4
done
