#!/bin/bash
# GPU box: full -m gpu suite, smoke, then one bench line. First failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/check
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -10 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
