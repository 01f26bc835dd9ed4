#!/bin/bash
# GPU box: the bench line (configs[2], the driver's --steps 20 --warmup 5 unless BENCH_ARGS says
# otherwise) under prover / NTT knobs, interleaved rounds on one box; prints proofs/s and ms/step.
# VARIANTS="name:ENV=.. ENV=..;name2:..."   ROUNDS (default 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
V="${VARIANTS:-base:}"
ARGS="${BENCH_ARGS:---steps 20 --warmup 5}"
for r in $(seq 1 "${ROUNDS:-3}"); do
  IFS=';' read -ra VS <<< "$V"
  for v in "${VS[@]}"; do
    name="${v%%:*}"; envs="${v#*:}"
    line=$(env $envs timeout -k 5 120 python3 bench.py --no-config5 --no-cpu-baseline $ARGS 2>/dev/null | tail -1) || { echo "variant $name failed"; exit 1; }
    echo "round $r $name $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(round(d['value']), round(d['ms_per_step'], 3))" "$line")"
  done
done
