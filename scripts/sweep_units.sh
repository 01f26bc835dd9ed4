#!/bin/bash
# lanes / unit-size sweep of bench.py (one process per configuration, each under its own limit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {
  echo -n "lanes=$1 unit=$2: "
  XFG_LANES=$1 XFG_UNIT=$2 timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${EXTRA:-} > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), round(d['ms_per_step'],2))" gpurun_out/sweep_$1_$2.json
}
for cfg in ${SWEEP:-4:16 4:8 4:32 3:16 6:16 6:8 8:8 2:32}; do run ${cfg%%:*} ${cfg##*:} || exit 1; done
