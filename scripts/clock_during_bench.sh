#!/bin/bash
# GPU box: shader clock and power sampled with rocm-smi while bench.py runs a long window (4000 steps, ~17 s):
# the clock the pipelined proving actually runs at (against the 2.4 GHz peak the VALU ceilings assume)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/clkb
timeout -k 10 300 python3 bench.py --steps 4000 --warmup 5 --no-cpu-baseline --no-config5 > gpurun_out/clkb/bench.json 2> gpurun_out/clkb/bench.err &
B=$!
for i in $(seq 1 60); do
  kill -0 $B 2>/dev/null || break
  echo "t=$SECONDS $(timeout 10 rocm-smi --showclocks --showpower 2>&1 | grep -E 'sclk|Socket Graphics Package Power' | tr -s ' ' | tr '\n' ' ')" >> gpurun_out/clkb/smi.txt
  sleep 0.5
done
wait $B; rc=$?
cat gpurun_out/clkb/smi.txt
python3 -c "import json; print(json.load(open('gpurun_out/clkb/bench.json'))['value'])"
exit $rc
