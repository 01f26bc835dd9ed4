#!/bin/bash
# GPU box: bench.py value and trace-LDE launch-set time of several builds (LIBS), REPS interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abl
for rep in $(seq 1 ${REPS:-3}); do
  for L in $LIBS; do
    XFG_LIB=$L timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 \
      > gpurun_out/abl/b.json 2> gpurun_out/abl/b.err || { tail -3 gpurun_out/abl/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abl/b.json')); print(sys.argv[1], round(d['value']), d['roofline']['kernel'].split(', ')[-2])" $L
  done
done
