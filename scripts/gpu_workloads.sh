# every bench workload at N=1 (each under its own limit), plus the VALU microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro_valu > gpurun_out/micro_valu.txt 2>&1 || { echo micro failed; exit 1; }
for w in cfg2 cfg3 cfg4 cfg5; do
  extra=""
  [ "$w" = cfg5 ] && extra="--steps 3 --warmup 1"
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline $extra > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/bench_$w.err; exit 1; }
  cut -c1-400 gpurun_out/bench_$w.json
done
