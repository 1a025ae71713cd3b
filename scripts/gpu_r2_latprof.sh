set -o pipefail
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r2/latprof -o run --output-format csv -- python3 scripts/lat_prof.py > gpurun_out/r2/latprof.txt 2>&1 || { tail -5 gpurun_out/r2/latprof.txt; exit 1; }
grep median gpurun_out/r2/latprof.txt
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r2/latprof/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 60 kernels: the tail of the table commits
for r in rows[-14:]:
    print(r["Kernel_Name"][:50], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us  start", int(r["Start_Timestamp"]) // 1000 % 100000000)
PY
