# end-of-session check on the final tree: whole GPU suite, smoke, default bench, cfg5 line
set -o pipefail
bash scripts/gpu_r2_final.sh || exit 1
timeout -k 10 400 python3 bench.py --workload cfg5 > gpurun_out/r2/final/cfg5.json 2> gpurun_out/r2/final/cfg5.err || { echo "cfg5 failed"; tail -5 gpurun_out/r2/final/cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2/final/cfg5.json')); print('cfg5', round(d['value'],1), round(d['ms_per_step'],3), d['parity']['ok'], round(d['secondary']['valu_roofline']['frac'],3), d['cpu_baseline']['value'])"
