# fixed-base path: parity tests, then bench variants (each GPU step under its own limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_fixed.py -x -q > gpurun_out/fixed_tests.log 2>&1; rc=$?
tail -5 gpurun_out/fixed_tests.log
[ $rc -eq 0 ] || { echo "fixed tests failed rc=$rc"; grep -E "^E |FAILED|Error" gpurun_out/fixed_tests.log | head -30; exit 1; }
for fb in ${FIXED_VARIANTS:-15 14 16}; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --fixed-bits $fb > gpurun_out/bench_fb$fb.json 2> gpurun_out/bench_fb$fb.err || { echo "bench fb=$fb failed"; tail -20 gpurun_out/bench_fb$fb.err; exit 1; }
  cut -c1-200 gpurun_out/bench_fb$fb.json
  python3 -c "import json;d=json.load(open('gpurun_out/bench_fb$fb.json'));print(d['config']['msm'], d['secondary'])"
done
