# round-2 measurement: Pippenger serial breakdown, default bench, and rocprof
# kernel stats of the serial (one stream: isolated kernel durations) and the
# default two-stream bench
set -o pipefail
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/pip_serial.json 2> gpurun_out/r2/pip_serial.err || { echo "pip serial failed"; tail -20 gpurun_out/r2/pip_serial.err; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || { echo "bench failed"; tail -20 gpurun_out/r2/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_serial -o run --output-format csv -- python3 bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r2/prof_serial.json 2> gpurun_out/r2/prof_serial.err || { echo "prof serial failed"; tail -20 gpurun_out/r2/prof_serial.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_pip -o run --output-format csv -- python3 bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/prof_pip.json 2> gpurun_out/r2/prof_pip.err || { echo "prof pip failed"; tail -20 gpurun_out/r2/prof_pip.err; exit 1; }
for d in prof_serial prof_pip; do f=$(find gpurun_out/r2/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; cut -d, -f1-8 "$f" | head -14; done
cat gpurun_out/r2/pip_serial.json gpurun_out/r2/bench.json
