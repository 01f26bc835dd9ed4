set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1 ; rc=$?
tail -5 gpurun_out/r4a/gputest.log
exit $rc
