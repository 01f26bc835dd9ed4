#!/bin/bash
# Round profile bundle (GPU box): bench line, rocprofv3 --kernel-trace --stats of the bench command,
# and separate PMC passes (FETCH_SIZE, WRITE_SIZE, VALU counts) on the trace-LDE launch sets alone,
# for configs[2] (64 proofs, 2^16 x 8: scripts/lde_only.py) and configs[4] (4 proofs = one config5 call, 2^20 x 16:
# scripts/lde_c5.py). Every GPU step runs under its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/round
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "rocprof trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5trace -o c5 -- python3 scripts/lde_c5.py 4 > $OUT/c5trace.log 2>&1 || { echo "c5 trace failed"; tail -5 $OUT/c5trace.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" VALUBusy OccupancyPercent; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python3 scripts/lde_only.py 64 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/c5pmc$i -o pmc -- python3 scripts/lde_c5.py 4 > $OUT/c5pmc$i.log 2>&1 || { echo "c5 pmc pass $i failed"; tail -5 $OUT/c5pmc$i.log; exit 1; }
done
python3 scripts/summarize_round.py $OUT
