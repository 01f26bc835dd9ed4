#!/bin/bash
# GPU-box script: bench line + rocprofv3 kernel stats (run via gpurun). Each GPU step bounded.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps ${STEPS:-3} --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
