#!/bin/bash
# GPU box: effective shader clock per kernel of one timing-mode 64-proof batch (scripts/stage_kernels.py):
# GRBM_GUI_ACTIVE (GPU busy cycles) / kernel duration from a --pmc pass (per-dispatch counters carry
# the dispatch's start / end) -- are isolated kernel durations taken at a lower clock than the pipeline's?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/clk
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/p -o pmc -- python3 ${STAGE_SCRIPT:-scripts/stage_kernels.py} > $OUT/p.log 2>&1 || { tail -5 $OUT/p.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])))
print(list(rows[0].keys()))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
durs = {}
for r in rows:
    key = (r["Dispatch_Id"], r["Kernel_Name"].split("(")[0])
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    if "Start_Timestamp" in r and r.get("End_Timestamp"):
        durs[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
per = collections.defaultdict(list)
for key, c in acc.items():
    d = durs.get(key)
    if d and c.get("GRBM_GUI_ACTIVE"):
        per[key[1]].append((c["GRBM_GUI_ACTIVE"] / d, c.get("GRBM_COUNT", 0) / d, d / 1e3))
for k, v in sorted(per.items(), key=lambda kv: -sum(x[2] for x in kv[1]))[:12]:
    v = v[-6:]
    print(f"{k[:50]:50s} GHz(gui_active/dur)={sum(x[0] for x in v)/len(v):5.2f} grbm_count/dur={sum(x[1] for x in v)/len(v):5.2f} dur_us={sum(x[2] for x in v)/len(v):8.1f}")
PY
