#!/bin/bash
# GPU box: bench.py at world size 1 without and with the RCCL exchange step (--dist under
# torch.distributed.run: one scatter of packed inputs per step, gather of fixed-size proof records),
# and with rank 0's N = EMUL exchange load (--dist --emulate-ranks EMUL, default 8: one RCCL gather
# per step receiving EMUL real-size records, the EMUL - 1 peer rows copied D2H), REPS interleaved
# rounds. XFG_BENCH_PHASES splits the --dist loops' host time (scatter / submit / wait / gather).
# EMUL_ENVS="A=1 B=2": also the emulated run under each of these environment settings (A/B of a knob).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dist
run_dist() {  # $1 = output tag, rest = extra bench args
  local tag=$1; shift
  XFG_BENCH_PHASES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps ${STEPS:-20} --warmup 3 \
    --no-cpu-baseline --no-config5 --dist "$@" > gpurun_out/dist/$tag.json 2>gpurun_out/dist/$tag.err \
    || { tail -3 gpurun_out/dist/$tag.err; exit 1; }
}
val() { python3 -c "import json,sys; print(round(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value']))" $1; }
for rep in $(seq 1 ${REPS:-3}); do
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/dist/a.json 2>/dev/null || exit 1
  run_dist b
  run_dist c --emulate-ranks ${EMUL:-8}
  extra=""
  for e in $EMUL_ENVS; do
    env $e bash -c "$(declare -f run_dist); run_dist d --emulate-ranks ${EMUL:-8}" || exit 1
    extra="$extra emul${EMUL:-8}[$e] $(val gpurun_out/dist/d.json)"
  done
  echo "plain $(val gpurun_out/dist/a.json) dist $(val gpurun_out/dist/b.json) dist+emul${EMUL:-8} $(val gpurun_out/dist/c.json)$extra"
  grep "phases ms" gpurun_out/dist/b.err | tail -1
  grep "phases ms" gpurun_out/dist/c.err | tail -1
done
