#!/bin/bash
# round 4: conflict-free pitch of the radix-32 split tiles (pitch, in-tree) vs the 64-bit pitch (cur):
# parity of the 2^20-point LDEs, LDS conflict cycles, LDE time per proof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "r1024 or tile_paths or large or config5" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
grep -cE "PASSED" $O/par.log; grep -E "FAILED|ERROR" $O/par.log
for L in cur pitch; do
  echo "== $L"; XFG_LIB=ab/$L.so bash scripts/pmc_lde.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES" | grep -E "ntt|CONFLICT|IDX|WAIT|CYCLES" || exit 1
done
LIBS="cur:ab/cur.so pitch:ab/pitch.so" ITERS=40 bash scripts/r4_c5lde.sh 2>&1 | grep -E "^==|proofs|gridY" || exit 1
