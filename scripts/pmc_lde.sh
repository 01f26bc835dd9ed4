#!/bin/bash
# NTT occupancy / VALU utilisation counters on the trace-LDE launch sets (one rocprofv3 --pmc pass per
# group, each under its own time limit; the first failure ends the script)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_lde
rm -rf $OUT && mkdir -p $OUT
i=0
for grp in "VALUBusy" "VALUUtilization" "OccupancyPercent" "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 $R/scripts/lde_only.py 64) > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "ntt_pass" not in k: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k[:60], {c: round(sum(v) / len(v), 2) for c, v in d.items()})
PY
