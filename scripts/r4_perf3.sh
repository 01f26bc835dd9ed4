#!/bin/bash
# round 4 (second session), first measurement pass on HEAD: bench line, configs[4] R=1024 kernels
# against the previous radix-32 passes (XFG_LIB A/B), exchange cost at world size 1, batch verify
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4p3
mkdir -p $O
[ -n "$SKIP_BENCH" ] || { timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }; }
[ -n "$SKIP_BENCH" ] || python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['roofline']['frac'], d['verify'], d['config5']['proofs_per_s'], d['config5']['trace_lde_1proof_ms'], d['config5']['trace_lde_ms'])"
AB="XFG_LIB=ab/cur.so XFG_LIB=ab/nor1024.so" bash scripts/c5_ab.sh 2>&1 | tee $O/c5ab.txt || exit 1
LIBS="cur:ab/cur.so nor1024:ab/nor1024.so" SHAPE=c5 REPS=1 bash scripts/lde_ab.sh > $O/lde_c5.txt 2>&1 || { tail $O/lde_c5.txt; exit 1; }
grep -E "^==|ntt_pass|launch-set" $O/lde_c5.txt
timeout -k 10 120 python3 scripts/verify_probe.py 64 5 2>&1 | tee $O/verify64.txt || exit 1
timeout -k 10 200 python3 scripts/verify_probe.py 512 3 2>&1 | tee $O/verify512.txt || exit 1
REPS=2 bash scripts/dist_ab.sh 2>&1 | tee $O/dist.txt || exit 1
