set -o pipefail
D=gpurun_out/r2/lat6
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_fixed.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/quick.log 2>&1 || { tail -30 $D/quick.log; exit 1; }
tail -1 $D/quick.log
for tag in pippenger table; do
  LAT_TAGS=$tag timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$tag -o run --output-format csv -- python3 scripts/lat_prof.py > $D/latprof_$tag.txt 2>&1 || { tail -5 $D/latprof_$tag.txt; exit 1; }
  grep median $D/latprof_$tag.txt
  python3 - $D/prof_$tag/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last call: from the last scalar upload (first copy after the previous call's last kernel)
last = rows[-40:]
t0 = None
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %-60s %8.1f us  gap %7.1f" % (r["Kernel_Name"][:60], (e - s) / 1e3, 0 if t0 is None else (s - t0) / 1e3))
    t0 = e
PY
done
