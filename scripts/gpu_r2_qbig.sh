# chip-wide single-opening quotient: parity, then the benchmark-common latency sweep
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_quotient_abi.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -k "quotient or single_opening or prove or multi_proof" --timeout 300 --timeout-method thread > gpurun_out/r2/tests_qbig.log 2>&1; rc=$?
tail -3 gpurun_out/r2/tests_qbig.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_qbig.log | head -30; exit $rc; }
timeout -k 10 600 python3 bench.py --workload common > gpurun_out/r2/common.json 2> gpurun_out/r2/common.err || { echo "common failed"; tail -20 gpurun_out/r2/common.err; exit 1; }
grep common: gpurun_out/r2/common.err
