# FETCH_SIZE calibration for the table's gather pattern, and the table path's
# traffic with the 80-B (default) and 64-B packed entries; one counter per pass
set -o pipefail
mkdir -p gpurun_out/r2/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r2/pmc/gather -o run --output-format csv -- ./scripts/micro_gather 32 67108864 > gpurun_out/r2/pmc/gather.txt 2>&1 || { echo "gather pmc failed"; tail -5 gpurun_out/r2/pmc/gather.txt; exit 1; }
grep -E "^k_" gpurun_out/r2/pmc/gather.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r2/pmc/fetch_l29 -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/pmc/fetch_l29.json 2> gpurun_out/r2/pmc/fetch_l29.err || { echo "l29 pmc failed"; tail -5 gpurun_out/r2/pmc/fetch_l29.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r2/pmc/write_l29 -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/pmc/write_l29.json 2> gpurun_out/r2/pmc/write_l29.err || { echo "l29 write pmc failed"; tail -5 gpurun_out/r2/pmc/write_l29.err; exit 1; }
export KZGX_LIB=variants/packed/libkzgx.so
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r2/pmc/fetch_packed -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/pmc/fetch_packed.json 2> gpurun_out/r2/pmc/fetch_packed.err || { echo "packed pmc failed"; tail -5 gpurun_out/r2/pmc/fetch_packed.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/bench_packed.json 2> gpurun_out/r2/bench_packed.err || { echo "packed bench failed"; tail -5 gpurun_out/r2/bench_packed.err; exit 1; }
unset KZGX_LIB
python3 - <<'PY'
import csv, collections, json
for d in ["gather", "fetch_l29", "write_l29", "fetch_packed"]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/r2/pmc/{d}/run_counter_collection.csv")):
        agg[(r["Kernel_Name"].split("(")[0][:50], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "gather" in d or "fixed_accum" in k[0] or "k_stream" in k[0]:
            print(d, k, len(v), "mean", sum(v) / len(v))
b = json.load(open("gpurun_out/r2/bench_packed.json"))
print("packed bench", b["value"], b["ms_per_step"], b["config"]["msm"], b["parity"])
PY
