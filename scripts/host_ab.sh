#!/bin/bash
# GPU box: bench.py value under host-side env variants (VARIANTS="name:ENV=..;.."), REPS interleaved
# rounds; then one short run with XFG_TRACE=1 whose per-unit host phase times are summarised
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hab
V="${VARIANTS:-base:}"
IFS=';' read -ra VS <<< "$V"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    name="${v%%:*}"; envs="${v#*:}"
    env $envs timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 \
      > gpurun_out/hab/b.json 2> gpurun_out/hab/b.err || { tail -3 gpurun_out/hab/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/hab/b.json')); print(sys.argv[1], round(d['value']))" $name
  done
done
if [ -n "$TRACE" ]; then
  XFG_TRACE=1 timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 > gpurun_out/hab/t.json 2> gpurun_out/hab/trace.err || exit 1
  python3 - <<'PY'
import re, collections
acc = collections.defaultdict(list)
for line in open("gpurun_out/hab/trace.err"):
    if not line.startswith("[xfg] B="): continue
    for k, v in re.findall(r" (\w+)=([0-9.]+)", line):
        acc[k].append(float(v))
for k, v in acc.items():
    v.sort()
    print(f"{k:14s} n={len(v):4d} mean={sum(v)/len(v):7.3f} p50={v[len(v)//2]:7.3f} p90={v[int(len(v)*0.9)]:7.3f}")
PY
fi
