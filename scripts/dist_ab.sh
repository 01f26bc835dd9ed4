#!/bin/bash
# GPU box: bench.py at world size 1 with and without the RCCL exchange step (--dist under
# torch.distributed.run: one scatter of packed inputs per step, gather of fixed-size proof records),
# REPS interleaved rounds -- the per-step cost of the exchange on rank 0; XFG_BENCH_PHASES splits the
# --dist loop's host time (scatter / submit / wait / gather)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dist
for rep in $(seq 1 ${REPS:-3}); do
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/dist/a.json 2>/dev/null || exit 1
  XFG_BENCH_PHASES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 --dist > gpurun_out/dist/b.json 2>gpurun_out/dist/b.err || { tail -3 gpurun_out/dist/b.err; exit 1; }
  python3 -c "import json; a=json.load(open('gpurun_out/dist/a.json')); b=json.loads(open('gpurun_out/dist/b.json').read().strip().splitlines()[-1]); print('plain', round(a['value']), 'dist', round(b['value']), 'verify gpu/host', a['verify']['gpu_proofs_per_s'], a['verify']['host_proofs_per_s'])"
  grep "phases ms" gpurun_out/dist/b.err | tail -1
done
