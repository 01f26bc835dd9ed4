#!/bin/bash
# GPU box: does the exchange's RCCL group cost the lanes a hardware queue? bench.py plain, --dist and
# --dist --emulate-ranks 8 at the default 4 hardware queues per process and with GPU_MAX_HW_QUEUES=5
# (one more queue for the exchange's side stream and RCCL's streams), REPS interleaved rounds, 20 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dq
val() { python3 -c "import json,sys; print(round(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value']))" $1; }
run() {  # tag, env, extra bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --dist "$@" \
    > gpurun_out/dq/$tag.json 2> gpurun_out/dq/$tag.err || { tail -3 gpurun_out/dq/$tag.err; exit 1; }
  echo -n "$tag $(val gpurun_out/dq/$tag.json)  "
}
for rep in $(seq 1 ${REPS:-3}); do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/dq/a.json 2>/dev/null || exit 1
  echo -n "plain $(val gpurun_out/dq/a.json)  "
  GPU_MAX_HW_QUEUES=5 timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/dq/a5.json 2>/dev/null || exit 1
  echo -n "plain_q5 $(val gpurun_out/dq/a5.json)  "
  run dist "X=1"
  run dist_q5 "GPU_MAX_HW_QUEUES=5"
  run emul8 "X=1" --emulate-ranks 8
  run emul8_q5 "GPU_MAX_HW_QUEUES=5" --emulate-ranks 8
  echo
done
