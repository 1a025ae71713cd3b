# packed-layout default: fixed tests (every window incl. 16/17), bench c=16 and c=17
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/tests_packed.log 2>&1; rc=$?
tail -3 gpurun_out/r2/tests_packed.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_packed.log | head -30; exit $rc; }
timeout -k 10 400 python3 bench.py --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/bench_c16.json 2> gpurun_out/r2/bench_c16.err || { echo "c16 failed"; tail -5 gpurun_out/r2/bench_c16.err; exit 1; }
timeout -k 10 400 python3 bench.py --fixed-bits 17 --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/bench_c17.json 2> gpurun_out/r2/bench_c17.err || { echo "c17 failed"; tail -5 gpurun_out/r2/bench_c17.err; exit 1; }
python3 -c "
import json
for f in ['c16','c17']:
    d = json.load(open('gpurun_out/r2/bench_%s.json' % f))
    print(f, d['value'], d['ms_per_step'], d['config']['msm'], d['parity'], d['roofline']['traffic'], d['secondary']['fixed_table_setup_s'], d['secondary']['valu_roofline']['frac'])
"
