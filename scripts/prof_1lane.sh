#!/bin/bash
# single-lane kernel profile of the proving pipeline (no cross-lane overlap in the durations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
XFG_LANES=1 XFG_UNIT=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o p1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { tail -5 gpurun_out/prof1.log; exit 1; }
f=$(find gpurun_out/prof1 -name "*kernel_trace.csv" | head -1)
python3 scripts/per_batch.py $f
