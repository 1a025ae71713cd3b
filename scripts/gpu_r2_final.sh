# whole GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r2/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/final/tests_all.log 2>&1; rc=$?
tail -3 gpurun_out/r2/final/tests_all.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/final/tests_all.log | head -30; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/final/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r2/final/smoke.log; exit 1; }
tail -1 gpurun_out/r2/final/smoke.log
timeout -k 10 500 python3 bench.py > gpurun_out/r2/final/bench.json 2> gpurun_out/r2/final/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2/final/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2/final/bench.json')); print(round(d['value']), d['ms_per_step'], d['parity'], round(d['secondary']['pippenger']['value']), d['roofline']['frac'], d['roofline']['traffic'], d['secondary']['valu_roofline']['frac'], d['cpu_baseline']['value'])"
