#!/bin/bash
# GPU box, round 5 first pass: the new -m gpu tests, then the exchange A/B at N = 8 load and the
# coherent-host-block A/B against the round-4 build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5a
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_dist.py "tests/test_gpu_parity.py::test_one_lane_back_to_back_units_match_oracle" \
  "tests/test_gpu_parity.py::test_gpu_batch_verify_node_vector_mutants" -k "not config3" > gpurun_out/r5a/tests.txt 2>&1 \
  || { tail -30 gpurun_out/r5a/tests.txt; exit 1; }
tail -3 gpurun_out/r5a/tests.txt
REPS=2 bash scripts/dist_ab.sh 2>&1 | tee gpurun_out/r5a/dist_ab.txt || exit 1
NO_LDE=1 REPS=2 LIBS="xfg-stark_amd/libxfgstark.so build/libxfgstark_r4.so" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/r5a/coherent_ab.txt
