#!/bin/bash
# A/B of environment knobs on the same box: bench.py once per setting (each under its own limit)
# usage: AB="XFG_UP_WMIN=1 XFG_UP_WMIN=64" bash scripts/ab_env.sh  (a comma joins variables of one setting)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
for kv in $AB; do
  echo -n "$kv (rep $rep): "
  env ${kv//,/ } timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), round(d['ms_per_step'],3), 'lde', d['roofline']['kernel'].split(', ')[-2])" gpurun_out/ab.json
done
done
