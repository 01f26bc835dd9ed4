#!/bin/bash
# GPU box: trace-LDE launch-set time (HIP events, xfg_bench_lde) under NTT tuning knobs, interleaved
# rounds on one box. SHAPE="count n blowup" (default configs[2]: 64 2^16 8);
# VARIANTS="name:ENV=.. ENV=..;name2:..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
read -r CNT N BL <<< "${SHAPE:-64 65536 8}"
V="${VARIANTS:-base:}"
for r in 1 2 3; do
  IFS=';' read -ra VS <<< "$V"
  for v in "${VS[@]}"; do
    name="${v%%:*}"; envs="${v#*:}"
    ms=$(env $envs timeout -k 5 90 python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver(); print(f'{p.bench_lde($CNT, $N, $BL, 10):.3f} ms')") || { echo "variant $name failed"; exit 1; }
    echo "round $r $name $ms"
  done
done
