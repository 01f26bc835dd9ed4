#!/bin/bash
# round 4: host-sequenced exchange -- the GPU tests of the sharded path, then --dist vs plain at world size 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 880 --timeout-method thread > $O/dist_tests.log 2>&1 || { tail -30 $O/dist_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/dist_tests.log
REPS=3 bash scripts/dist_ab.sh 2>&1 | tee $O/dist.txt || exit 1
