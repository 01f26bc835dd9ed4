#!/bin/bash
# GPU box: bench.py --steps 20 --warmup 5 at several pipeline depths (batches in flight), 3 interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dab
for rep in 1 2 3; do
  for d in 4 6 8 10; do
    timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --depth $d --no-cpu-baseline --no-config5 > gpurun_out/dab/b.json 2> gpurun_out/dab/b.err || { tail -3 gpurun_out/dab/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/dab/b.json')); print('depth', sys.argv[1], round(d['value']))" $d
  done
done
