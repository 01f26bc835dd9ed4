#!/bin/bash
# GPU box (round 5): BLAKE3 with its xor (and add) in the VOP3 encoding -- compression ubench, isolated
# kernel durations of one 64-proof batch, and bench proofs/s, against the current build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/b3
for b in b3_ubench b3_ubench_x64 b3_ubench_xa64; do echo "== $b"; timeout -k 10 60 ./scripts/ubench/$b || exit 1; done 2>&1 | tee gpurun_out/b3/ubench.txt
VARIANTS="r5:XFG_X=0;b3x:XFG_LIB=build/libxfgstark_b3x.so;b3xa:XFG_LIB=build/libxfgstark_b3xa.so" ROUNDS=2 bash scripts/kt_ab.sh 2>&1 | head -20 | tee gpurun_out/b3/kt_ab.txt || exit 1
NO_LDE=1 REPS=2 LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_b3x.so build/libxfgstark_b3xa.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/b3/lib_ab.txt
