set -o pipefail
bash scripts/gpu_tests_all.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print('cfg2', round(d['value']), d['secondary']['valu_roofline'])"
timeout -k 10 400 python bench.py --workload cfg5 --steps 5 --warmup 2 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { tail -10 gpurun_out/bench_cfg5.err; exit 1; }
cat gpurun_out/bench_cfg5.json
