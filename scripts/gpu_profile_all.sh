# round profile refresh: default bench (with CPU baseline), rocprof kernel stats,
# PMC traffic passes, and the other workloads; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out/prof gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cut -c1-300 gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { echo "prof failed"; tail -20 gpurun_out/prof_bench.err; exit 1; }
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $pmc -d gpurun_out/pmc/$pmc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --serial > gpurun_out/pmc_$pmc.json 2> gpurun_out/pmc_$pmc.err || { echo "pmc $pmc failed"; tail -5 gpurun_out/pmc_$pmc.err; exit 1; }
done
for w in cfg3 cfg4; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 1; }
  cut -c1-200 gpurun_out/bench_$w.json
done
timeout -k 10 400 python bench.py --workload cfg5 --steps 3 --warmup 1 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { tail -20 gpurun_out/bench_cfg5.err; exit 1; }
cut -c1-200 gpurun_out/bench_cfg5.json
