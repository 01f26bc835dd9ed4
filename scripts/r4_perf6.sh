#!/bin/bash
# round 4: configs[4] pass A seeds from small tables (seed) and tile-pair block order (seedpair, in-tree):
# parity of the 2^20-point LDEs, then LDE time per proof and traffic against the previous build (cur)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "r1024 or tile_paths or large or config5" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
grep -cE "PASSED" $O/par.log; grep -E "FAILED|ERROR" $O/par.log
LIBS="cur:ab/cur.so seed:ab/seed.so seedpair:ab/seedpair.so" ITERS=40 bash scripts/r4_c5lde.sh 2>&1 | grep -E "^==|proofs|gridY" || exit 1
LIBS="cur:ab/cur.so seed:ab/seed.so seedpair:ab/seedpair.so" SHAPE=c5 ARGS="1 20 16 40" REPS=1 bash scripts/lde_ab.sh > $O/lde_c5.txt 2>&1 || { tail $O/lde_c5.txt; exit 1; }
grep -E "^==|ntt_pass|launch-set" $O/lde_c5.txt
