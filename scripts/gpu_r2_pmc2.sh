# DRAM read requests by size (32/64/128 B) for the gather calibration and both table layouts
set -o pipefail
mkdir -p gpurun_out/r2/pmc2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/r2/pmc2/gather -o run --output-format csv -- ./scripts/micro_gather 32 67108864 > gpurun_out/r2/pmc2/gather.txt 2>&1 || { echo "gather pmc failed"; tail -5 gpurun_out/r2/pmc2/gather.txt; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc $P -d gpurun_out/r2/pmc2/l29 -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/pmc2/l29.json 2> gpurun_out/r2/pmc2/l29.err || { echo "l29 pmc failed"; tail -5 gpurun_out/r2/pmc2/l29.err; exit 1; }
KZGX_LIB=variants/packed/libkzgx.so timeout -s KILL 200 rocprofv3 --pmc $P -d gpurun_out/r2/pmc2/packed -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/pmc2/packed.json 2> gpurun_out/r2/pmc2/packed.err || { echo "packed pmc failed"; tail -5 gpurun_out/r2/pmc2/packed.err; exit 1; }
python3 - <<'PY'
import csv, collections
for d in ["gather", "l29", "packed"]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/r2/pmc2/{d}/run_counter_collection.csv")):
        agg[(r["Kernel_Name"].split("(")[0][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        if "gather" in d or "fixed_accum" in k[0] or "k_stream" in k[0]:
            print(d, k, len(v), "mean %.0f" % (sum(v) / len(v)))
PY
