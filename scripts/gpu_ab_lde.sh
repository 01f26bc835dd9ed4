#!/bin/bash
# GPU box: NTT parity tests, then same-box A/B of an env knob (AB="K=0 K=1") on the trace-LDE launch
# set (64 proofs, 30 reps) and on bench.py proofs/s, alternating settings; every step bounded
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/ablde
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
lde() {
  env $1 timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); p.prepare(64, 1 << 16); print(round(p.bench_lde(64, 1 << 16, 8, 30), 4))"
}
for rep in 1 2; do
  for kv in $AB; do echo -n "$kv lde ms: "; lde $kv || exit 1; done
done
for rep in 1 2; do
  for kv in $AB; do
    echo -n "$kv: "
    env $kv timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > $OUT/ab.json 2> $OUT/ab.err || { tail -3 $OUT/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), round(d['ms_per_step'],3), 'lde', d['roofline']['kernel'].split(', ')[-2])" $OUT/ab.json
  done
done
