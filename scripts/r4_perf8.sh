#!/bin/bash
# round 4: configs[4] pass A with the t-independent [k1][j2] four-step table (tab4, in-tree) vs the running product (cur):
# parity of the 2^20-point LDEs, counters, LDE time per proof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "r1024 or tile_paths or large or config5" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
grep -cE "PASSED" $O/par.log; grep -E "FAILED|ERROR" $O/par.log
for L in cur tab4; do
  echo "== $L"; XFG_LIB=ab/$L.so bash scripts/pmc_lde.sh "SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" FETCH_SIZE | grep -E "ntt|VALU|WAIT|CYCLES|FETCH" || exit 1
done
LIBS="cur:ab/cur.so tab4:ab/tab4.so" ITERS=40 bash scripts/r4_c5lde.sh 2>&1 | grep -E "^==|proofs|gridY" || exit 1
