# benchmark-common: degree-2^23 commit test, then the latency sweep over a 10,429,000-point setup
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k benchmark_common --timeout 250 --timeout-method thread > gpurun_out/r2/tests_common.log 2>&1; rc=$?
tail -3 gpurun_out/r2/tests_common.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_common.log | head -30; exit $rc; }
timeout -k 10 600 python3 bench.py --workload common > gpurun_out/r2/common.json 2> gpurun_out/r2/common.err || { echo "common failed"; tail -20 gpurun_out/r2/common.err; exit 1; }
grep common: gpurun_out/r2/common.err
python3 -c "import json; d=json.load(open('gpurun_out/r2/common.json')); print(d['secondary']['setup_s'], d['parity'])"
