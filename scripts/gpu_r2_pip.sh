# Pippenger redesign: parity (everything that runs the table-less MSM), then the serial Pippenger bench + rocprof
set -o pipefail
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
true || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_sharded_abi.py tests/test_gpu_cpp_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/tests_pip.log 2>&1; rc=$?
tail -4 gpurun_out/r2/tests_pip.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/tests_pip.log | head -30; exit $rc; }
for v in main; do
  if [ $v = main ]; then unset KZGX_LIB; else export KZGX_LIB=variants/$v/libkzgx.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_pip_$v -o run --output-format csv -- python3 bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/prof_pip_$v.json 2> gpurun_out/r2/prof_pip_$v.err || { echo "prof pip failed"; tail -20 gpurun_out/r2/prof_pip_$v.err; exit 1; }
done
unset KZGX_LIB
timeout -k 10 300 python bench.py --fixed-bits 0 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2/pip2.json 2> gpurun_out/r2/pip2.err || { echo "pip failed"; tail -20 gpurun_out/r2/pip2.err; exit 1; }
python3 - <<'PY'
import csv, json
for v in ["main"]:
    print("==", v)
    for r in csv.DictReader(open(f"gpurun_out/r2/prof_pip_{v}/run_kernel_stats.csv")):
        if "msm" in r["Name"]:
            print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:10.1f}')
    d = json.load(open(f"gpurun_out/r2/prof_pip_{v}.json"))
    print(v, d["value"], d["ms_per_step"], d.get("parity"))
d = json.load(open(f"gpurun_out/r2/pip2.json"))
print("2-stream", d["value"], d["ms_per_step"], d.get("parity"), d["secondary"].get("latency"))
PY
