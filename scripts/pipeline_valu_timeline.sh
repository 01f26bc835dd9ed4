#!/bin/bash
# GPU box: kernel trace of the pipelined bench + per-kernel VALU instruction counts (separate --pmc
# run of the same command) -> VALU issue demand over time (scripts/valu_timeline.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/vtl
rm -rf $OUT && mkdir -p $OUT
(cd /tmp && env ${EXTRA//,/ } timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-config5) > $OUT/t.log 2>&1 || { echo "trace failed"; tail -5 $OUT/t.log; exit 1; }
(cd /tmp && env ${EXTRA//,/ } timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/p -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config5) > $OUT/p.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p.log; exit 1; }
python3 $R/scripts/valu_timeline.py $OUT
