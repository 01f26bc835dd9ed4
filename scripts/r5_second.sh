#!/bin/bash
# GPU box, round 5 second pass: LDE parity on the new R = 1024 addressing, configs[4] LDE A/B
# against the round-4 build, the exchange experiment, the VALU micro-benchmark and the VALU ledger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5b
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "lde or r1024 or 2p20 or interpolat" > gpurun_out/r5b/tests.txt 2>&1 || { tail -30 gpurun_out/r5b/tests.txt; exit 1; }
tail -2 gpurun_out/r5b/tests.txt
LIBS="r5:xfg-stark_amd/libxfgstark.so st8:build/libxfgstark_st8.so r4:build/libxfgstark_r4.so" SHAPE=c5 REPS=2 bash scripts/lde_ab.sh > gpurun_out/r5b/c5_lde_ab.txt 2>&1 || { tail -5 gpurun_out/r5b/c5_lde_ab.txt; exit 1; }
grep "==" gpurun_out/r5b/c5_lde_ab.txt
timeout -k 10 60 ./scripts/ubench/valu_ubench > gpurun_out/r5b/valu_ubench.txt || exit 1
bash scripts/valu_ledger.sh > gpurun_out/r5b/valu_ledger.txt 2>&1 || { tail -5 gpurun_out/r5b/valu_ledger.txt; exit 1; }
bash scripts/r5_exexp.sh 2>&1 | tee gpurun_out/r5b/exexp.txt
