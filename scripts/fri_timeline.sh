#!/bin/bash
# GPU box: the ordered kernels of the last of 3 timing-mode 64-proof batches (2^16 x 8, one stream),
# from the DEEP LDE to the end of the batch, with the idle gap before each kernel: where the FRI
# stage's time goes (kernel time vs gaps between launches and copies)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/fritl
rm -rf $OUT && mkdir -p $OUT
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace ${API:+--hip-runtime-trace} --output-format csv -d $OUT/t -o t -- python3 $OLDPWD/scripts/stage_kernels.py) > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
grep "{" $OUT/log
python3 - $OUT <<'PY'
import csv, glob, sys
d = sys.argv[1]
ev = []
for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
mc = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
if mc:
    for r in csv.DictReader(open(mc[0])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
ev.sort()
ks = [i for i, e in enumerate(ev) if not e[2].startswith("copy")]
last = ev[ks[2 * len(ks) // 3]:]  # roughly the last batch
# from the last forward LDE pass B (the DEEP LDE) on
ib = max(i for i, e in enumerate(last) if "ntt_pass_b_tq" in e[2])
seq = last[ib:]
t0, prev = seq[0][0], seq[0][1]
busy = 0
for s, e, k in seq:
    gap = max(0, s - prev)
    busy += (e - s)
    print(f"{(s - t0) / 1e3:8.1f} us  +gap {gap / 1e3:6.1f}  dur {(e - s) / 1e3:7.1f}  {k}")
    prev = max(prev, e)
print(f"span {(seq[-1][1] - t0) / 1e3:.0f} us, busy {busy / 1e3:.0f} us, {len(seq)} events")
# host side: the HIP API calls of the same window and how long each took
ht = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)
if ht:
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", ""))
                 for r in csv.DictReader(open(ht[0])))
    w0, w1 = seq[0][0] - 3000_000, seq[-1][1]
    for s, e, f, tid in api:
        if w0 <= s <= w1 and (e - s) > 20_000:
            print(f"api {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  {f}  tid {tid}")
PY
