#!/bin/bash
# GPU box: PMC of the trace-LDE launch sets alone at 2^16 x 8 (64 proofs) and 2^20 x 16 (1 proof):
# VALU instructions, stall split (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY of WAVE_CYCLES), LDS
# bank conflicts, VALUBusy, HBM bytes; one rocprofv3 pass per counter group, per-kernel means
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/ldecmp
rm -rf $OUT && mkdir -p $OUT
PROG="import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
p = xfgstark.XfgBurnMintProver()
print('c2', p.bench_lde(64, 1 << 16, 8, 3)); print('c5', p.bench_lde(1, 1 << 20, 16, 3))"
i=0
for grp in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "VALUBusy" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 -c "$PROG" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
grep -h "^c[25]" $OUT/p1.log
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if "ntt" in k:
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
