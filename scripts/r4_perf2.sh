#!/bin/bash
# round 4, second perf pass: parity of the new 2^20 kernels, configs[4] LDE variants; exchange variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r4p2
for L in ab/r1024.so ab/r1024chunk.so; do
  XFG_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "r1024 or tile_paths or large_traces" > gpurun_out/r4p2/par_$(basename $L).log 2>&1 || { tail -20 gpurun_out/r4p2/par_$(basename $L).log; exit 1; }
  tail -1 gpurun_out/r4p2/par_$(basename $L).log
done
LIBS="cf:ab/cf.so pair:ab/pair.so r1024:ab/r1024.so r1024chunk:ab/r1024chunk.so" SHAPE=c5 REPS=2 bash scripts/lde_ab.sh > gpurun_out/r4p2/lde_c5.txt 2>&1 || { tail gpurun_out/r4p2/lde_c5.txt; exit 1; }
grep -E "^==|lde_ms|launch-set|ntt_pass" gpurun_out/r4p2/lde_c5.txt | grep -v "calls=   28" | head -60
for v in "XFG_EXCHANGE_PRIO=0" "XFG_EXCHANGE_THREAD=1" "XFG_EXCHANGE_PRIO=1" "XFG_EXCHANGE_THREAD=1 XFG_EXCHANGE_PRIO=1 XFG_EXCHANGE_SLOTS=6"; do
  echo "== $v"
  env $v XFG_BENCH_PHASES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --dist > gpurun_out/r4p2/d.json 2>gpurun_out/r4p2/d.err || { tail -3 gpurun_out/r4p2/d.err; exit 1; }
  python3 -c "import json; b=json.loads(open('gpurun_out/r4p2/d.json').read().strip().splitlines()[-1]); print('dist', round(b['value']))"
  grep "phases ms" gpurun_out/r4p2/d.err | tail -1
done
timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/r4p2/a.json 2>/dev/null || exit 1
python3 -c "import json; a=json.load(open('gpurun_out/r4p2/a.json')); print('plain', round(a['value']))"
