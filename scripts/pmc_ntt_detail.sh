#!/bin/bash
# GPU box: wave-state counters of the trace-LDE passes (where the wave cycles go), one pass per group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_ntt
rm -rf $OUT && mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && env ${EXTRA//,/ } timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 $R/scripts/${SCRIPT:-lde_only.py} 64) > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k)
    for c in sorted(m): print(f"    {c:24s} {m[c]:.4g}")
PY
