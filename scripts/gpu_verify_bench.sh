set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_cpp_api.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > gpurun_out/verify_tests.log 2>&1; rc=$?
tail -3 gpurun_out/verify_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/verify_tests.log | head -20; exit 1; }
for c in BN254 BLS12381; do
timeout -k 10 300 python scripts/bench_verify.py --curve $c > gpurun_out/verify_bench_$c.json 2> gpurun_out/verify_bench_$c.err || { tail -10 gpurun_out/verify_bench_$c.err; exit 1; }
cat gpurun_out/verify_bench_$c.json
done
