#!/bin/bash
# GPU box: isolated kernel durations of one 64-proof batch in timing mode (scripts/stage_kernels.py
# under rocprofv3 --kernel-trace) per knob variant, interleaved rounds; scripts/kt_ab_summary.py
# prints the mean duration per kernel of the 64-proof launches. VARIANTS="name:ENV=..;name2:.."; STAGE_SCRIPT
# another timing-mode script (scripts/stage_kernels_c5.py: one configs[4] call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
V="${VARIANTS:-base:}"
OUT=gpurun_out/kt_ab
rm -rf $OUT && mkdir -p $OUT
for r in $(seq 1 "${ROUNDS:-2}"); do
  IFS=';' read -ra VS <<< "$V"
  for v in "${VS[@]}"; do
    name="${v%%:*}"; envs="${v#*:}"
    env $envs timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name.$r -o kt -- python3 ${STAGE_SCRIPT:-scripts/stage_kernels.py} > $OUT/$name.$r.log 2>&1 || { echo "variant $name failed"; tail -3 $OUT/$name.$r.log; exit 1; }
  done
done
python3 scripts/kt_ab_summary.py $OUT
