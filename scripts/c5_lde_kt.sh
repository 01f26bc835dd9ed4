#!/bin/bash
# GPU box: rocprofv3 kernel trace of the configs[4] trace-LDE launch sets alone (1 proof, 7 columns,
# 2^20 x 16), per-kernel stats; then the PMC comparison of scripts/lde_pmc_cmp.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/c5kt
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/lde_c5.py 1 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
grep " ms" $OUT/kt.log
python3 scripts/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 12
bash scripts/lde_pmc_cmp.sh
