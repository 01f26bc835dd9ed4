#!/bin/bash
# multi-lane kernel trace of bench.py + GPU busy analysis (union of kernel intervals)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profb -o pb -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/profb.log 2>&1 || { tail -5 gpurun_out/profb.log; exit 1; }
f=$(find gpurun_out/profb -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_busy.py $f > gpurun_out/busy.txt
head -40 gpurun_out/busy.txt
XFG_TRACE=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/trace.log 2>&1
tail -30 gpurun_out/trace.log
