# round-2: new config tests, then full GPU suite, then default bench
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_quotient_abi.py tests/test_gpu_sharded_abi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/tests_new.log 2>&1; rc=$?
tail -5 gpurun_out/r2/tests_new.log
[ $rc -eq 0 ] || { echo "new tests failed rc=$rc"; grep -E "^E |FAILED|Error" gpurun_out/r2/tests_new.log | head -30; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || { echo "bench failed"; tail -20 gpurun_out/r2/bench.err; exit 1; }
cat gpurun_out/r2/bench.json
