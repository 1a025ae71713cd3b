# the whole GPU suite (what the driver runs at round end), time-limited
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/tests_all.log 2>&1; rc=$?
tail -8 gpurun_out/tests_all.log
[ $rc -eq 0 ] || grep -E "FAILED|Error|error" gpurun_out/tests_all.log | head -30
exit $rc
