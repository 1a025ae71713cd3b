# verify-half GPU parity (pairing, G2 MSM, verify_proof); each step time-limited
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pairing_tests.log 2>&1; rc=$?
tail -25 gpurun_out/pairing_tests.log
exit $rc
