#!/bin/bash
# GPU box, round 5 third pass: the whole -m gpu suite, bench proofs/s against the round-4 build, and
# rank 0's emulated N = 8 exchange load (own row on the host; rows copied D2H per step or left in HBM)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5c
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r5c/tests.txt 2>&1 || { tail -40 gpurun_out/r5c/tests.txt; exit 1; }
tail -2 gpurun_out/r5c/tests.txt
NO_LDE=1 REPS=2 LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_r4.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/r5c/lib_ab.txt || exit 1
bash scripts/r5_exexp.sh 2>&1 | tee gpurun_out/r5c/exexp.txt
