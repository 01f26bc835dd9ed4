#!/bin/bash
# GPU box (round 5): BLAKE3 half-rounds as fixed-order asm blocks (scripts/b3_sched_gen.py) --
# smoke on the default build, then isolated kernel durations of one 64-proof batch for the five
# schedules (s0 = default, s1..s4 = XFG_B3_SCHED) and the compiler-scheduled rounds (cs); STAGE=bench
# compares bench proofs/s instead; STAGE=occ the default (alt / s_nop after fast) against volatile
# half-rounds (v), 5 waves per SIMD for the leaf kernels (w5), both (vw5) and cs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/b3s
L="s0:XFG_X=0;s1:XFG_LIB=build/libxfgstark_s1.so;s2:XFG_LIB=build/libxfgstark_s2.so;s3:XFG_LIB=build/libxfgstark_s3.so;s4:XFG_LIB=build/libxfgstark_s4.so;cs:XFG_LIB=build/libxfgstark_cs.so"
if [ "$STAGE" = occ ]; then
  NO_LDE=1 REPS=${REPS:-2} LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_w5.so build/libxfgstark_v.so build/libxfgstark_vw5.so build/libxfgstark_cs.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/b3s/occ_ab.txt
  exit $?
fi
if [ "$STAGE" = bench ]; then
  NO_LDE=1 REPS=${REPS:-2} LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_s1.so build/libxfgstark_s2.so build/libxfgstark_s3.so build/libxfgstark_cs.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/b3s/lib_ab.txt
  exit $?
fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3 | tee gpurun_out/b3s/smoke.txt || exit 1
VARIANTS="$L" ROUNDS=2 bash scripts/kt_ab.sh 2>&1 | head -24 | tee gpurun_out/b3s/kt_ab.txt
