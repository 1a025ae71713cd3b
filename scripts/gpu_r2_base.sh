# round-2 baseline: Pippenger breakdown (serial + 2-stream), single-call latencies
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2/pip_serial.json 2> gpurun_out/r2/pip_serial.err || { echo "pip serial failed"; tail -20 gpurun_out/r2/pip_serial.err; exit 1; }
timeout -k 10 300 python bench.py --fixed-bits 0 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2/pip.json 2> gpurun_out/r2/pip.err || { echo "pip failed"; tail -20 gpurun_out/r2/pip.err; exit 1; }
timeout -k 10 300 python scripts/latency.py 0 > gpurun_out/r2/lat_pip.json 2> gpurun_out/r2/lat_pip.err || { echo "lat failed"; tail -20 gpurun_out/r2/lat_pip.err; exit 1; }
timeout -k 10 300 python scripts/latency.py 16 > gpurun_out/r2/lat_fixed.json 2> gpurun_out/r2/lat_fixed.err || { echo "lat16 failed"; tail -20 gpurun_out/r2/lat_fixed.err; exit 1; }
cat gpurun_out/r2/*.json
