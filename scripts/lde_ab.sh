#!/bin/bash
# GPU box: trace-LDE launch set (64 proofs, 30 reps) under each env setting in AB, interleaved 3x
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2 3; do
  for kv in $AB; do
    echo -n "$kv: "
    env ${kv//,/ } timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); p.prepare(64, 1 << 16); print(round(p.bench_lde(64, 1 << 16, 8, 30), 4))" || exit 1
  done
done
