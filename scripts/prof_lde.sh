#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lde -o lde -- python3 scripts/lde_bench.py > gpurun_out/prof_lde.log 2>&1 || { tail -20 gpurun_out/prof_lde.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_lde/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.2f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
