#!/bin/bash
# GPU box: same-box A/B of two builds of libxfgstark.so (XFG_LIB): the trace-LDE launch set
# (xfg_bench_lde, 64 proofs) and bench.py proofs/s, alternating A and B; each run bounded.
# LIBS="a.so b.so c.so" compares more builds, NO_LDE=1 skips the LDE timing, REPS (default 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
A=${A:-xfg-stark_amd/libxfgstark.so}
B=${B:-build/libxfgstark_b.so}
lde() {
  XFG_LIB=$1 timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); p.prepare(64, 1 << 16); print(round(p.bench_lde(64, 1 << 16, 8, 30), 4))"
}
LIBS=${LIBS:-$A $B}
if [ -z "$NO_LDE" ]; then
  for rep in 1 2; do
    for L in $LIBS; do echo -n "$L lde ms: "; lde $L || exit 1; done
  done
fi
for rep in $(seq 1 ${REPS:-2}); do
  for L in $LIBS; do
    echo -n "$L proofs/s: "
    XFG_LIB=$L timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 \
      > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err || { tail -3 gpurun_out/ab_lib.err; exit 1; }
    python3 -c "import json; print(round(json.load(open('gpurun_out/ab_lib.json'))['value']))"
  done
done
