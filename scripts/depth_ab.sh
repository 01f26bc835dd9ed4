#!/bin/bash
# GPU box: DFT occupancy micro-benchmark, then bench.py at submission depth 2 / 3 / 4 (each run bounded)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -x build/dft_v2 ]; then timeout -k 5 60 ./build/dft_v2 || exit 1; fi
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), round(d['ms_per_step'],3))" "$1"; }
for d in ${DEPTHS:-2 3 4}; do
  echo -n "depth $d steps ${STEPS:-20}: "
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 --depth $d \
    > gpurun_out/depth$d.json 2> gpurun_out/depth$d.err || { tail -3 gpurun_out/depth$d.err; exit 1; }
  show gpurun_out/depth$d.json
done
