#!/bin/bash
# GPU box: bench.py proofs/s of several builds of libxfgstark.so (LIBS="a.so b.so ..."), REPS
# interleaved rounds, each run bounded; prints per-build mean and spread
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abb
: > gpurun_out/abb/res.txt
for rep in $(seq 1 ${REPS:-4}); do
  for L in $LIBS; do
    env ${ENVS//,/ } XFG_LIB=$L timeout -k 10 240 python3 bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --no-config5 \
      > gpurun_out/abb/b.json 2> gpurun_out/abb/b.err || { tail -3 gpurun_out/abb/b.err; exit 1; }
    v=$(python3 -c "import json; print(round(json.load(open('gpurun_out/abb/b.json'))['value']))")
    echo "$L $v" | tee -a gpurun_out/abb/res.txt
  done
done
python3 - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for l in open("gpurun_out/abb/res.txt"):
    k, v = l.split(); d[k].append(float(v))
for k, v in d.items():
    print(f"{k:40s} mean {statistics.mean(v):8.0f}  sd {statistics.pstdev(v):6.0f}  n {len(v)}")
PY
