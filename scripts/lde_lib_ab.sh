#!/bin/bash
# GPU box: the trace-LDE launch sets alone (xfg_bench_lde, HIP events: 64 proofs of 2^16 x 8 over 110
# sets, 4 proofs of 2^20 x 16 over 36 sets) for several library builds (LIBS), REPS interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for rep in $(seq 1 ${REPS:-3}); do
  for L in $LIBS; do
    XFG_LIB=$L timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver()
print(sys.argv[1], 'c2 %.4f ms' % p.bench_lde(64, 1 << 16, 8, 110), 'c5 %.4f ms' % p.bench_lde(4, 1 << 20, 16, 36))" $L || exit 1
  done
done
