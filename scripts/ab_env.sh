#!/bin/bash
# A/B of environment knobs on the same box: bench.py once per setting (each under its own limit)
# usage: AB="XFG_UP_WMIN=1 XFG_UP_WMIN=64" bash scripts/ab_env.sh  (a comma joins variables of one setting)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
: > gpurun_out/ab_res.txt
for rep in $(seq 1 ${REPS:-2}); do
for kv in $AB; do
  env ${kv//,/ } timeout -k 10 240 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-config5 ${BARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '(rep ' + sys.argv[3] + '):', round(d['value']), round(d['ms_per_step'],3), 'lde', d['roofline']['kernel'].split(', ')[-2])" gpurun_out/ab.json "$kv" "$rep" | tee -a gpurun_out/ab_res.txt
done
done
python3 - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_res.txt"):
    k, rest = l.split(" (rep ", 1) if " (rep " in l else (None, None)
    if k: d[k].append(float(rest.split("): ")[1].split()[0]))
for k, v in d.items():
    print(f"{k:40s} mean {statistics.mean(v):8.0f}  sd {statistics.pstdev(v):6.0f}  n {len(v)}")
PY
