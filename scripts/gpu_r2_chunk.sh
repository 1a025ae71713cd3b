# single large MSM: chunked (default) vs one un-chunked Pippenger, benchmark-common sweep + 2^20 parity
set -o pipefail
mkdir -p gpurun_out/r2/chunk
unset KZGX_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q -k "cfg5_commit_single or benchmark_common or large_single" --timeout 250 --timeout-method thread > gpurun_out/r2/chunk/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/chunk/tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/chunk/tests.log | head -20; exit $rc; }
timeout -k 10 600 python3 bench.py --workload common > gpurun_out/r2/chunk/common_final.json 2> gpurun_out/r2/chunk/common_final.err || { echo "common failed"; tail -20 gpurun_out/r2/chunk/common_final.err; exit 1; }
grep common: gpurun_out/r2/chunk/common_final.err
