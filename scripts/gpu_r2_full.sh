# round-2: whole GPU suite (new config tests first), then a serial rocprof run of the default bench
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/tests_all.log 2>&1; rc=$?
tail -8 gpurun_out/r2/tests_all.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_all.log | head -30; exit $rc; }
