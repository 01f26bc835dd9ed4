#!/bin/bash
# GPU box: kernel durations of the configs[4]-size interpolations (scripts/interp_c5.py) per build
# (LIBS="name:path ..."), one rocprofv3 --kernel-trace run each, mean per pass kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/interp
rm -rf $OUT && mkdir -p $OUT
for v in ${LIBS:-base:xfg-stark_amd/libxfgstark.so}; do
  name=${v%%:*}; lib=${v#*:}
  XFG_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o kt -- python3 scripts/interp_c5.py > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
  python3 - $OUT/$name $name <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])):
    acc[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    if "ntt_pass" in k:
        print(f"{sys.argv[2]:6s} {k:45s} n={len(v):3d} us: " + " ".join(f"{x:.0f}" for x in v))
PY
done
