#!/bin/bash
# GPU box: same-box A/B of the configs[4] side measurement (2^20-step trace LDE at blowup 16 and
# proofs/s of 4-proof quadratic-extension batches, bench.config5), alternating settings
# usage: AB="XFG_LIB=ab/liba.so XFG_LIB=ab/libb.so" bash scripts/c5_ab.sh   (any env setting works;
# a comma joins several variables into one setting: XFG_LIB=ab/liba.so,XFG_LANES=6)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for kv in $AB; do
    echo -n "$kv: "
    env ${kv//,/ } timeout -k 10 180 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); sys.path.insert(0, '.')
import torch; torch.cuda.init()
import xfgstark, bench
p = xfgstark.XfgBurnMintProver()
c5 = bench.config5(p, 0)
print('c5 proofs/s', c5['proofs_per_s'], 'trace lde ms', c5['trace_lde_ms'])" || exit 1
  done
done
