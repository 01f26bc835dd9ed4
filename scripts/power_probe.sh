#!/bin/bash
# GPU box: board power / clocks sampled while bench.py runs (is the proving loop power-capped?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/power
rm -rf $OUT && mkdir -p $OUT
(timeout -k 10 200 python3 bench.py --steps ${STEPS:-3000} --warmup 3 --no-cpu-baseline --no-config5 > $OUT/bench.json 2> $OUT/bench.err) &
BP=$!
for i in $(seq 1 40); do
  timeout 20 rocm-smi --showpower --showclocks 2>&1 | grep -E "Socket|sclk" | tr -s ' ' | tr '\n' ' ' >> $OUT/smi.txt
  echo >> $OUT/smi.txt
  sleep 0.5
  kill -0 $BP 2>/dev/null || break
done
wait $BP
cat $OUT/smi.txt
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'])"
