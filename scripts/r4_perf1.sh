#!/bin/bash
# round 4, first perf pass: exchange A/B, configs[4] LDE A/B (coset-consecutive pass A order), bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4p1
REPS=2 bash scripts/dist_ab.sh 2>&1 | tee gpurun_out/r4p1/dist.txt || exit 1
LIBS="base:ab/base.so cf:ab/cf.so" SHAPE=c5 REPS=2 bash scripts/lde_ab.sh 2>&1 | tee gpurun_out/r4p1/lde_c5.txt || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4p1/bench.json 2> gpurun_out/r4p1/bench.err || { tail -5 gpurun_out/r4p1/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4p1/bench.json')); print(d['value'], d['roofline']['frac'], d['verify'], d['config5']['proofs_per_s'], d['config5']['trace_lde_1proof_ms'], d['config5']['trace_lde_ms'])"
