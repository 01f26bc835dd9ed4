#!/bin/bash
# GPU box (round 5): a BLAKE3 schedule change (first: half-rounds specialised on known-zero message words, the add3 of a zero
# padding word as a two-source e64 add; then round 1's diagonal half as a block) -- the -m gpu suite on the tree's build, then bench proofs/s
# against the previous commit (head) and the compiler-scheduled rounds (cs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/b3z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/b3z/gputest.log 2>&1; rc=$?
tail -2 gpurun_out/b3z/gputest.log
[ $rc = 0 ] || exit $rc
NO_LDE=1 REPS=${REPS:-3} LIBS="${LIBS:-xfg-stark_amd/libxfgstark.so build/libxfgstark_head.so build/libxfgstark_cs.so}" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/b3z/lib_ab.txt
