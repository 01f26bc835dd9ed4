#!/bin/bash
# GPU box: same-box A/B of two bench.py trees at the driver's settings (--steps 20 --warmup 5),
# alternating; usage: A=abl/old/bench.py B=bench.py bash scripts/bench_ab.sh  (the library is the
# in-tree build for both: XFG_LIB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export XFG_LIB=$PWD/xfg-stark_amd/libxfgstark.so
for rep in $(seq 1 ${REPS:-3}); do
  for b in $A $B; do
    timeout -k 10 240 python3 $b --steps ${STEPS:-20} --warmup ${WARM:-5} --no-cpu-baseline --no-config5 > gpurun_out/bab.json 2> gpurun_out/bab.err || { tail -3 gpurun_out/bab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/bab.json $b
  done
done
