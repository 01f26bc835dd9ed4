#!/bin/bash
# lanes / guided-unit sweep of bench.py (one process per configuration, each under its own limit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {
  echo "lanes=$1 unit_max=$2 unit_min=$3"
  XFG_LANES=$1 XFG_UNIT=$2 XFG_UNIT_MIN=$3 timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${EXTRA:-} > gpurun_out/sweep_$1_$2_$3.json 2> gpurun_out/sweep_$1_$2_$3.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), round(d['ms_per_step'],2))" gpurun_out/sweep_$1_$2_$3.json
}
run 4 16 16 && run 4 16 4 && run 4 16 8 && run 4 8 2 && run 6 16 4 && run 6 8 4 && run 8 8 4 && run 4 32 4
