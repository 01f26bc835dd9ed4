#!/bin/bash
# GPU box, a round's final bundle: the round profile (bench line, kernel traces, LDE PMC of both
# shapes: scripts/profile_round.sh), the whole-proof VALU ledger, the configs[1] single-proof kernel
# trace, smoke() and the no-flag default bench, on the final build. Then, on the CPU container,
# scripts/copy_bundle.sh rNN copies the results into profiles/rNN.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/profile_round.sh > gpurun_out/bundle.log 2>&1 || { tail -20 gpurun_out/bundle.log; exit 1; }
tail -5 gpurun_out/bundle.log
bash scripts/valu_ledger.sh > gpurun_out/valu_ledger.txt 2>&1 || { tail -5 gpurun_out/valu_ledger.txt; exit 1; }
rm -rf gpurun_out/single
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/single -o single -- python3 scripts/single_proof.py 10 gpurun_out/single/calls.txt > gpurun_out/single.log 2>&1 || { tail -5 gpurun_out/single.log; exit 1; }
python3 scripts/single_proof.py --summary gpurun_out/single > gpurun_out/single_summary.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -5 gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['whole_proof']['frac'], (d.get('config5') or {}).get('proofs_per_s'), d['single_proof']['ms'])"
