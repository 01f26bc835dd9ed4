set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lde or interpolate or ntt_edge or config5 or large_traces or quadratic" > gpurun_out/r2b/pytest.log 2>&1 || { tail -30 gpurun_out/r2b/pytest.log; exit 1; }
tail -2 gpurun_out/r2b/pytest.log
for e in 5 4 5 4; do echo "== XFG_NTT_E=$e"; XFG_NTT_E=$e timeout -k 10 120 python3 scripts/c5_stages.py 4 | head -12; done
