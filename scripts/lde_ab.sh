#!/bin/bash
# GPU box: same-box A/B of library builds (XFG_LIB) on the trace-LDE launch sets alone -- per-kernel
# durations (rocprofv3 --kernel-trace --stats) and HBM traffic (FETCH_SIZE, WRITE_SIZE: separate
# --pmc passes), REPS interleaved rounds.
# usage: LIBS="base:ab/base.so new:ab/new.so" SHAPE=c5|c2 bash scripts/lde_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
SHAPE=${SHAPE:-c5}
if [ "$SHAPE" = c5 ]; then ARGS=${ARGS:-"1 20 16 5"}; else ARGS=${ARGS:-"64 16 8 5"}; fi
PROG="import sys; sys.path.insert(0, 'xfg-stark_amd'); import xfgstark
a = [int(x) for x in '$ARGS'.split()]
p = xfgstark.XfgBurnMintProver()
print('lde_ms', round(p.bench_lde(a[0], 1 << a[1], a[2], a[3]), 4))"
for rep in $(seq 1 ${REPS:-2}); do
  for lv in $LIBS; do
    name=${lv%%:*}; lib=${lv#*:}
    OUT=gpurun_out/ldeab/$name.$rep
    rm -rf $OUT && mkdir -p $OUT
    XFG_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -c "$PROG" > $OUT/kt.log 2>&1 || { echo "$name kt failed"; tail -5 $OUT/kt.log; exit 1; }
    echo "== $name rep $rep: $(grep lde_ms $OUT/kt.log)"
    python3 scripts/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 4
    if [ "$rep" = 1 ]; then
      for c in FETCH_SIZE WRITE_SIZE; do
        XFG_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o pmc -- python3 -c "$PROG" > $OUT/$c.log 2>&1 || { echo "$name $c failed"; tail -5 $OUT/$c.log; exit 1; }
      done
      python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*_SIZE/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
tot = 0.0
for k, d in sorted(acc.items()):
    if "ntt_pass" in k:
        m = {c: sum(v) / len(v) for c, v in d.items()}
        # gfx950: FETCH_SIZE counts 64 B requests as 32 B -- doubled per MI355X_MICROARCH.md
        b = 2 * m.get("FETCH_SIZE", 0) * 1024 + m.get("WRITE_SIZE", 0) * 1024
        tot += b
        print(f"  {k:48s} fetch_kB={m.get('FETCH_SIZE', 0):12.0f} write_kB={m.get('WRITE_SIZE', 0):12.0f} traffic_GB={b / 1e9:.3f}")
print(f"  launch-set traffic (sum of per-kernel means) {tot / 1e9:.3f} GB")
PY
    fi
  done
done
