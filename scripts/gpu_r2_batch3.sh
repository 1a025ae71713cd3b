# fold/finish split: Pippenger parity + serial profile; then the table-path decomposition sweep
set -o pipefail
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pippenger_buckets.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/tests_b3.log 2>&1; rc=$?
tail -2 gpurun_out/r2/tests_b3.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_b3.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_pip3 -o run --output-format csv -- python3 bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/prof_pip3.json 2> gpurun_out/r2/prof_pip3.err || { echo "prof failed"; tail -5 gpurun_out/r2/prof_pip3.err; exit 1; }
python3 - <<'PY'
import csv, json
for r in csv.DictReader(open("gpurun_out/r2/prof_pip3/run_kernel_stats.csv")):
    if "msm" in r["Name"]:
        print(f'{r["Name"][:50]:50s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:9.1f}')
d = json.load(open("gpurun_out/r2/prof_pip3.json")); print("pip serial", round(d["value"]), round(d["ms_per_step"], 3))
PY
timeout -k 10 300 python3 bench.py --fixed-bits 0 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2/pip3.json 2> gpurun_out/r2/pip3.err || { echo "pip failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2/pip3.json')); print('pip 2-stream', round(d['value']), round(d['ms_per_step'],3), d['secondary']['latency']['pippenger']['commit_ms'])"
bash scripts/gpu_r2_ppt.sh
