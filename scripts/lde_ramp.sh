#!/bin/bash
# GPU box: per-launch-set durations over a long back-to-back window of trace-LDE launch sets
# (rocprofv3 kernel trace): shows how long the first launch sets after an idle GPU run slow
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ramp
rm -rf $O && mkdir -p $O
ARGS=${ARGS:-"64 16 8 120"}
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 -c "
import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
a = [int(x) for x in '$ARGS'.split()]
p = xfgstark.XfgBurnMintProver()
print('lde_ms', round(p.bench_lde(a[0], 1 << a[1], a[2], a[3]), 4))" > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
grep lde_ms $O/log
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
ev = [e for e in ev if "ntt_pass" in e[2]]
sets = [(ev[i][0], ev[i + 1][1], (ev[i][1] - ev[i][0]) / 1e3, (ev[i + 1][1] - ev[i + 1][0]) / 1e3) for i in range(0, len(ev) - 1, 2)]
t0 = sets[0][0]
for k, (s, e, a, b) in enumerate(sets):
    if k < 12 or k % 10 == 0 or k == len(sets) - 1:
        print(f"set {k:3d} t={(s - t0) / 1e6:7.2f} ms  A {a:7.1f} us  B {b:7.1f} us  set {(e - s) / 1e3:7.1f} us")
PY
