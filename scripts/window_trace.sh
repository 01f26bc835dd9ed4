#!/bin/bash
# GPU box: kernel trace of one default-shape bench window (20 timed steps after 5 warmup steps) and,
# per 2 ms of the timed window, the fraction of time any kernel runs and the mean number of kernels
# in flight: where the window's fixed fill / drain cost sits (scripts/window_trace.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/wtrace
rm -rf $OUT && mkdir -p $OUT
(cd /tmp && XFG_BENCH_TIMELINE=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 $OLDPWD/bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-config5) > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
grep -E "^\{|timeline" $OUT/log | cut -c1-300
python3 scripts/window_trace.py $OUT | tee $OUT/summary.txt
