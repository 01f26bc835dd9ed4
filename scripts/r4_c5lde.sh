#!/bin/bash
# round 4: configs[4] trace LDE per proof at 1 / 2 / 4 proofs per launch set, library builds A/B (LIBS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/c5lde
rm -rf $O && mkdir -p $O
for rep in 1 2; do
  for lv in ${LIBS:-cur:xfg-stark_amd/libxfgstark.so}; do
    name=${lv%%:*}; lib=${lv#*:}
    echo "== $name rep $rep"
    XFG_LIB=$lib timeout -k 10 120 python3 scripts/lde_scale.py 1 2 4 || exit 1
  done
done
for lv in ${LIBS:-cur:xfg-stark_amd/libxfgstark.so}; do
  name=${lv%%:*}; lib=${lv#*:}
  XFG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o kt -- python3 scripts/lde_scale.py 1 4 > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_Y"])) for r in csv.DictReader(open(f)))
ev = [e for e in ev if "ntt_pass" in e[2]]
prev = None
from collections import defaultdict
acc = defaultdict(list)
gaps = defaultdict(list)
for s, e, k, gy in ev:
    acc[(k[:40], gy)].append((e - s) / 1e3)
    if prev and prev[3] == gy:
        gaps[gy].append((s - prev[1]) / 1e3)
    prev = (s, e, k, gy)
for (k, gy), v in sorted(acc.items()):
    v = v[2:] if len(v) > 4 else v
    print(f"  {k:40s} gridY {gy:4d} n={len(v):3d} avg_us {sum(v)/len(v):9.1f} min {min(v):9.1f}")
for gy, g in sorted(gaps.items()):
    print(f"  gridY {gy}: launch gap avg {sum(g)/len(g):.1f} us")
PY
done
