#!/bin/bash
# GPU box, round 5: -m gpu suite on the e64-encoded BLAKE3 / shift forms, then bench proofs/s and the
# LDE launch sets against the previous commit's build (c1) and round 4 (r4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5d
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r5d/tests.txt 2>&1 || { tail -40 gpurun_out/r5d/tests.txt; exit 1; }
tail -2 gpurun_out/r5d/tests.txt
NO_LDE=1 REPS=2 LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_c1.so build/libxfgstark_r4.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/r5d/lib_ab.txt || exit 1
LIBS="new:xfg-stark_amd/libxfgstark.so c1:build/libxfgstark_c1.so" SHAPE=c2 REPS=2 bash scripts/lde_ab.sh > gpurun_out/r5d/c2_lde_ab.txt 2>&1 || exit 1
grep -E "^lde_ms|pass_" gpurun_out/r5d/c2_lde_ab.txt | grep -v fetch
