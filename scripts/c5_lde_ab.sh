#!/bin/bash
# GPU box: configs[4] trace-LDE launch set (1 proof, 7 columns, 2^20 x 16) under NTT tuning knobs,
# interleaved rounds on one box: VARIANTS="name:ENV=.. ENV=..;name2:..." (default: knob sweep)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
V="${VARIANTS:-base:;lta8:XFG_NTT_LTA=8;lta8preg:XFG_NTT_LTA=8 XFG_NTT_PREG=1;preg:XFG_NTT_PREG=1;ltb9:XFG_NTT_LTB=9;e4:XFG_NTT_E=4}"
for r in 1 2 3; do
  IFS=';' read -ra VS <<< "$V"
  for v in "${VS[@]}"; do
    name="${v%%:*}"; envs="${v#*:}"
    ms=$(env $envs timeout -k 5 60 python3 scripts/lde_c5.py 1) || { echo "variant $name failed"; exit 1; }
    echo "round $r $name $ms"
  done
done
