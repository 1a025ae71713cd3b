# default config (BN254 c=17 packed table): full bench, serial rocprof kernel stats, and the
# request-size PMC pass for roofline.traffic
set -o pipefail
mkdir -p gpurun_out/r2/def
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 python3 bench.py > gpurun_out/r2/def/bench.json 2> gpurun_out/r2/def/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2/def/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/def/prof_serial -o run --output-format csv -- python3 bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/def/prof_serial.json 2> gpurun_out/r2/def/prof_serial.err || { echo "prof failed"; tail -5 gpurun_out/r2/def/prof_serial.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/def/prof_2s -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/def/prof_2s.json 2> gpurun_out/r2/def/prof_2s.err || { echo "prof 2s failed"; tail -5 gpurun_out/r2/def/prof_2s.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/r2/def/pmc_rd -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/def/pmc_rd.json 2> gpurun_out/r2/def/pmc_rd.err || { echo "pmc failed"; tail -5 gpurun_out/r2/def/pmc_rd.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r2/def/pmc_wr -o run --output-format csv -- python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/def/pmc_wr.json 2> gpurun_out/r2/def/pmc_wr.err || { echo "pmc wr failed"; tail -5 gpurun_out/r2/def/pmc_wr.err; exit 1; }
python3 - <<'PY'
import csv, collections, json
for d in ["prof_serial", "prof_2s"]:
    for r in csv.DictReader(open(f"gpurun_out/r2/def/{d}/run_kernel_stats.csv")):
        if "fixed" in r["Name"] or "quotient" in r["Name"]:
            print(d, r["Name"][:48], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
for d in ["pmc_rd", "pmc_wr"]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/r2/def/{d}/run_counter_collection.csv")):
        if "fixed_accum" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, len(v), "mean %.0f" % (sum(v) / len(v)))
for f in ["bench", "prof_serial", "prof_2s"]:
    b = json.load(open(f"gpurun_out/r2/def/{f}.json"))
    print(f, round(b["value"]), round(b["ms_per_step"], 3), b["config"]["msm"], b["parity"]["ok"], b["roofline"]["avg_launch_ms"])
PY
