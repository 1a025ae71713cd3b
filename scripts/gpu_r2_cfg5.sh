# device-resident sharded commit: g1_sum_device test, C++ facade test, cfg5 bench at 1 GPU
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cpp_api.py -m gpu -x -q -k "g1_sum or cpp_api" --timeout 120 --timeout-method thread > gpurun_out/r2/tests_cfg5.log 2>&1; rc=$?
tail -3 gpurun_out/r2/tests_cfg5.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_cfg5.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --workload cfg5 --steps 10 --warmup 2 > gpurun_out/r2/cfg5.json 2> gpurun_out/r2/cfg5.err || { echo "cfg5 failed"; tail -20 gpurun_out/r2/cfg5.err; exit 1; }
cat gpurun_out/r2/cfg5.json
