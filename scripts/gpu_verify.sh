# verify-half GPU tests: pairing parity + C++ facade (testing.cpp port incl. verify/export)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_cpp_api.py -x -v --timeout 600 --timeout-method thread > gpurun_out/verify_tests.log 2>&1; rc=$?
tail -25 gpurun_out/verify_tests.log
[ $rc -eq 0 ] || grep -E "FAILED|Error|error" gpurun_out/verify_tests.log | head -30
exit $rc
