#!/bin/bash
# GPU box: isolated per-kernel durations of one batch in timing mode (one stream), the last of REPS:
# 64 proofs at 2^16 x 8 (scripts/stage_kernels.py, 3 batches), or PROG=scripts/c5_stages.py REPS=2 for
# configs[4] (4 proofs at 2^20 x 16, quadratic extension)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/stagek
rm -rf $OUT && mkdir -p $OUT
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o t -- python3 $OLDPWD/${PROG:-scripts/stage_kernels.py}) > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
grep "{" $OUT/log
python3 - $OUT ${REPS:-3} <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
# the last 1/REPS of the kernels = the last batch
reps = int(sys.argv[2])
third = [e for e in ev if e[0] >= ev[(reps - 1) * len(ev) // reps][0]]
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, k in third:
    agg[k][0] += 1; agg[k][1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
span = (third[-1][1] - third[0][0]) / 1e3
print(f"kernels {len(third)}  sum {tot:.0f} us  span {span:.0f} us")
for k, (c, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:24]:
    print(f"{us:9.1f} us  x{c:3d}  {k[:90]}")
PY
