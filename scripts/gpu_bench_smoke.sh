set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_small.json 2> gpurun_out/b_small.err || { echo small failed; tail -20 gpurun_out/b_small.err; exit 1; }
cat gpurun_out/b_small.json
timeout -k 10 600 python bench.py > gpurun_out/b_full.json 2> gpurun_out/b_full.err || { echo full failed; tail -20 gpurun_out/b_full.err; exit 1; }
cat gpurun_out/b_full.json
