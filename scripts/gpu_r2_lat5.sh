set -o pipefail
mkdir -p gpurun_out/r2/lat5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/lat5/quick.log 2>&1 || { tail -30 gpurun_out/r2/lat5/quick.log; exit 1; }
timeout -k 10 120 python3 scripts/lat_micro.py > gpurun_out/r2/lat5/lat_micro.txt 2>&1 || { tail -20 gpurun_out/r2/lat5/lat_micro.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r2/lat5/lat_micro.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fixed.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_pairing.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/lat5/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r2/lat5/tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r2/lat5/tests.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/lat5/prof -o run --output-format csv -- python3 scripts/lat_prof.py > gpurun_out/r2/lat5/latprof.txt 2>&1 || { tail -5 gpurun_out/r2/lat5/latprof.txt; exit 1; }
grep median gpurun_out/r2/lat5/latprof.txt
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r2/lat5/prof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-7:]:
    print(r["Kernel_Name"][:50], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
timeout -k 10 200 python3 scripts/vw_timing.py 2>&1 | tail -1
