# rocprofv3 kernel trace + stats of a short bench run (no PMC)
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { echo "prof failed"; tail -20 gpurun_out/prof_bench.err; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -30
