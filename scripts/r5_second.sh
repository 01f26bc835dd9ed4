#!/bin/bash
# GPU box, round 5 second pass: the -m gpu suite on the new field multiply / LDE addressing (all but
# the 8-rank configs[3] test), the LDE launch-set A/Bs (configs[4] and configs[2]) against the
# round-4 build and the A/B variants, the VALU micro-benchmark and the whole-proof VALU ledger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5b
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  -k "not config3" > gpurun_out/r5b/tests.txt 2>&1 || { tail -40 gpurun_out/r5b/tests.txt; exit 1; }
tail -2 gpurun_out/r5b/tests.txt
LIBS="r5:xfg-stark_amd/libxfgstark.so mulv1:build/libxfgstark_mulv1.so st8:build/libxfgstark_st8.so r4:build/libxfgstark_r4.so" \
  SHAPE=c5 REPS=2 bash scripts/lde_ab.sh > gpurun_out/r5b/c5_lde_ab.txt 2>&1 || { tail -5 gpurun_out/r5b/c5_lde_ab.txt; exit 1; }
grep "==" gpurun_out/r5b/c5_lde_ab.txt
LIBS="r5:xfg-stark_amd/libxfgstark.so mulv1:build/libxfgstark_mulv1.so r4:build/libxfgstark_r4.so" SHAPE=c2 REPS=2 \
  bash scripts/lde_ab.sh > gpurun_out/r5b/c2_lde_ab.txt 2>&1 || { tail -5 gpurun_out/r5b/c2_lde_ab.txt; exit 1; }
grep "==" gpurun_out/r5b/c2_lde_ab.txt
timeout -k 10 60 ./scripts/ubench/valu_ubench > gpurun_out/r5b/valu_ubench.txt || exit 1
bash scripts/valu_ledger.sh > gpurun_out/r5b/valu_ledger.txt 2>&1 || { tail -5 gpurun_out/r5b/valu_ledger.txt; exit 1; }
tail -25 gpurun_out/r5b/valu_ledger.txt
