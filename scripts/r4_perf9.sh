#!/bin/bash
# round 4: configs[4] intermediate in tile-major layout (tm, in-tree) vs row-major (cur):
# parity of the 2^20-point LDEs, counters, LDE time per proof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "r1024 or tile_paths or large or config5" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
grep -cE "PASSED" $O/par.log; grep -E "FAILED|ERROR" $O/par.log
for L in cur tm; do
  echo "== $L"; XFG_LIB=ab/$L.so bash scripts/pmc_lde.sh "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" FETCH_SIZE WRITE_SIZE | grep -E "ntt|WAIT|CYCLES|SIZE" || exit 1
done
LIBS="cur:ab/cur.so tm:ab/tm.so" ITERS=40 bash scripts/r4_c5lde.sh 2>&1 | grep -E "^==|proofs|gridY" || exit 1
