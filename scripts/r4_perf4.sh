#!/bin/bash
# round 4: exchange-step variants at world size 1 (bench.py --dist under torch.distributed.run) against
# the plain loop, interleaved; then a kernel trace of one --dist run (RCCL kernels and copies vs prover).
# Ran against the round-3 exchange of commit 4965fcf, whose XFG_EXCHANGE_* knobs are gone since d190dfe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4p4
mkdir -p $O
dist() {  # env settings..., then bench --dist
  env "$@" XFG_BENCH_PHASES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --dist > $O/d.json 2>$O/d.err || { tail -3 $O/d.err; return 1; }
  python3 -c "import json; b=json.loads(open('$O/d.json').read().strip().splitlines()[-1]); print('dist $*', round(b['value']))"
  grep "phases ms" $O/d.err | tail -1
}
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > $O/a.json 2>/dev/null || exit 1
  python3 -c "import json; a=json.load(open('$O/a.json')); print('plain', round(a['value']))"
  dist XFG_X=0 || exit 1
  dist XFG_EXCHANGE_THREAD=1 || exit 1
  dist XFG_EXCHANGE_PRIO=1 || exit 1
  dist XFG_EXCHANGE_THREAD=1 XFG_EXCHANGE_PRIO=1 || exit 1
done
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o kt -- python3 \
    bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-config5 --dist > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 scripts/kstats.py $(find $O/kt -name "*kernel_stats.csv" | head -1) 25
find $O/kt -name "*memory_copy_stats.csv" -exec cat {} \;
