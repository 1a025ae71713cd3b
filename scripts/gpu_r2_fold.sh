set -o pipefail
D=gpurun_out/r2/fold
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_pippenger_buckets.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/quick.log 2>&1 || { tail -30 $D/quick.log; exit 1; }
tail -1 $D/quick.log
timeout -k 10 120 python3 scripts/lat_micro.py > $D/lat_micro.txt 2>&1 || { tail -20 $D/lat_micro.txt; exit 1; }
grep -v amdgpu.ids $D/lat_micro.txt
LAT_TAGS=pippenger timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_pip -o run --output-format csv -- python3 scripts/lat_prof.py > $D/latprof_pip.txt 2>&1 || { tail -5 $D/latprof_pip.txt; exit 1; }
grep median $D/latprof_pip.txt
python3 - $D/prof_pip/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
for r in rows[-10:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %-60s %8.1f us  gap %7.1f" % (r["Kernel_Name"][:60], (e - s) / 1e3, 0 if t0 is None else (s - t0) / 1e3))
    t0 = e
PY
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $D/cfg2.json 2> $D/cfg2.err || { tail -20 $D/cfg2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$D/cfg2.json').read().strip().splitlines()[-1]); s=d['secondary']
print('cfg2', round(d['value']), {k: v for k, v in s.items() if 'pip' in k or 'latency' in k})"
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 10 --warmup 2 --no-cpu-baseline --no-latency > $D/cfg4.json 2> $D/cfg4.err || { tail -20 $D/cfg4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$D/cfg4.json').read().strip().splitlines()[-1]); s=d['secondary']
print('cfg4', round(d['value']), {k: v for k, v in s.items() if 'pip' in k or 'valu' in k or 'mixed' in k})"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -2 $D/tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $D/tests.log | head -30; exit $rc; }
