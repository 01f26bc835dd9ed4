#!/bin/bash
# GPU box: bench.py --steps 20 --warmup 5 (one rank) unpinned, pinned to the GPU's local NUMA node's
# CPUs, and pinned to the other node's CPUs (taskset, CPU lists from bench.gpu_local_cpus), REPS rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/numa
LOCAL=$(python3 -c "import bench; s=sorted(bench.gpu_local_cpus(0)); print(','.join(map(str,s)))")
REMOTE=$(python3 -c "import bench, os; s=sorted(set(os.sched_getaffinity(0)) - bench.gpu_local_cpus(0)); print(','.join(map(str,s)))")
for rep in $(seq 1 ${REPS:-3}); do
  for mode in none local remote; do
    case $mode in none) pre="";; local) pre="taskset -c $LOCAL";; remote) pre="taskset -c $REMOTE";; esac
    timeout -k 10 240 $pre python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config5 > gpurun_out/numa/b.json 2> gpurun_out/numa/b.err || { tail -3 gpurun_out/numa/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/numa/b.json')); print(sys.argv[1], round(d['value']), d['single_proof']['ms'])" $mode
  done
done
