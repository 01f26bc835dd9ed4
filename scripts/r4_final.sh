#!/bin/bash
# round 4, final pass on the final build: the -m gpu suite, the profile bundle (bench line, kernel trace,
# PMC of both trace-LDE shapes), the configs[4] depth sweep; every GPU step bounded, first failure ends it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_tests.sh || exit 1
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/profile_round.sh > gpurun_out/round_stdout.txt 2>&1 || { tail -20 gpurun_out/round_stdout.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/round/summary.json')); b=d; print('bundle', round(d['bench_value']), d['bench_roofline']['frac'], d['rocprof_lde_launch_set']['sum_ms'], d['lde_pmc_c5.json']['traffic_over_algorithmic'], d['bench_config5']['proofs_per_s'], d['bench_config5']['trace_lde_1proof_ms'])"
[ -n "$NO_DEPTH" ] || timeout -k 10 600 python3 scripts/c5_depth.py 4:4 4:6 4:8 2:8 8:4 8:6 4:4 || exit 1
