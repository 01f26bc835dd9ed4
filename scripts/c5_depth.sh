#!/bin/bash
# GPU box: configs[4] side measurement (bench.config5) at several batch / calls / depth settings
# usage: SETS="4,5,2 4,8,4" bash scripts/c5_depth.sh   (batch,calls,depth per setting)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for st in ${SETS:-4,5,2 4,8,4 8,4,2 2,10,4}; do
    IFS=, read b c d <<< "$st"
    echo -n "batch $b calls $c depth $d: "
    timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); sys.path.insert(0, '.')
import xfgstark, bench
p = xfgstark.XfgBurnMintProver()
c5 = bench.config5(p, $b, $c, $d)
print('c5 proofs/s', c5['proofs_per_s'])" || exit 1
  done
done
