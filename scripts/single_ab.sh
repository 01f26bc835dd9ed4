#!/bin/bash
# GPU box: `-m gpu`, then BASELINE configs[1] (one 2^16 proof, synchronous) best-of-20 for two builds
# alternating (A, B: XFG_LIB paths; default ab/pre.so against the in-tree library), then the in-tree
# build's single-proof kernel trace split by call (scripts/single_proof.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
A=${A:-ab/pre.so}
B=${B:-xfg-stark_amd/libxfgstark.so}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_sp_tests.txt 2>&1 || { tail -20 gpurun_out/r6_sp_tests.txt; exit 1; }
tail -1 gpurun_out/r6_sp_tests.txt
for rep in 1 2 3; do
  for L in $A $B; do
    echo -n "$L "; XFG_LIB=$L timeout -k 10 120 python3 scripts/single_proof.py 20 "" 2>&1 | grep "single proof" || exit 1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/single -o single -- python3 scripts/single_proof.py 10 gpurun_out/single/calls.txt > gpurun_out/single.log 2>&1 || { tail -5 gpurun_out/single.log; exit 1; }
python3 scripts/single_proof.py --summary gpurun_out/single > gpurun_out/single_summary.txt
