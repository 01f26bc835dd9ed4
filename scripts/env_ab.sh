#!/bin/bash
# GPU box: same-box sweep of the library's tuning knobs on the headline bench (bench.py --steps 20
# --warmup 3, no CPU baseline / configs[4] side measurement), settings interleaved, REPS rounds.
# usage: SETS="XFG_LANES=7 XFG_LANES=8 XFG_UNIT=16,XFG_SPLIT_MIN=8" bash scripts/env_ab.sh
# (a comma joins several variables into one setting; "-" = the defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for kv in $SETS; do
    [ "$kv" = "-" ] && e="" || e=${kv//,/ }
    echo -n "$kv: "
    env $e timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 \
      > gpurun_out/env_ab.json 2> gpurun_out/env_ab.err || { tail -3 gpurun_out/env_ab.err; exit 1; }
    python3 -c "import json; print(round(json.load(open('gpurun_out/env_ab.json'))['value']))"
  done
done
