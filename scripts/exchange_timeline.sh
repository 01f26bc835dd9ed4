#!/bin/bash
# GPU box: the timed window's step submissions and completions (XFG_BENCH_TIMELINE: host ms from the
# window start) for the plain loop, --dist at world size 1 and --dist --emulate-ranks 8, REPS rounds:
# where the exchange's fixed per-window cost sits (first scatter before the first submission, last
# gather after the last completion)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/extl
common="--steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5"
for rep in $(seq 1 ${REPS:-2}); do
  XFG_BENCH_TIMELINE=1 timeout -k 10 240 python3 bench.py $common > gpurun_out/extl/a.json 2> gpurun_out/extl/a.err || exit 1
  for tag in dist emul8; do
    extra=""; [ $tag = emul8 ] && extra="--emulate-ranks 8"
    XFG_BENCH_TIMELINE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 $common --dist $extra \
      > gpurun_out/extl/$tag.json 2> gpurun_out/extl/$tag.err || { tail -3 gpurun_out/extl/$tag.err; exit 1; }
  done
  for tag in a dist emul8; do
    f=gpurun_out/extl/$tag
    v=$(python3 -c "import json,sys; print(round(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value']))" $f.json)
    echo "$tag $v"
    grep -E "^(timeline|submitted) ms" $f.err | tail -2 | cut -c1-200
  done
done
