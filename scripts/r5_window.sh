#!/bin/bash
# GPU box (diagnostic): the exchange's cost per step vs per window -- plain, --dist and the emulated
# N = 8 load at 20 and at 300 timed steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/win
val() { python3 -c "import json,sys; print(round(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value']))" $1; }
for rep in 1 2; do
  for st in 20 300; do
    timeout -k 10 240 python3 bench.py --steps $st --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/win/a.json 2>/dev/null || exit 1
    for e in 0 8; do
      timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --gpus 1 --steps $st --warmup 3 --no-cpu-baseline --no-config5 --dist --emulate-ranks $e > gpurun_out/win/d$e.json 2>gpurun_out/win/d$e.err || { tail -3 gpurun_out/win/d$e.err; exit 1; }
    done
    echo "steps $st: plain $(val gpurun_out/win/a.json) dist $(val gpurun_out/win/d0.json) emul8 $(val gpurun_out/win/d8.json)"
  done
done
