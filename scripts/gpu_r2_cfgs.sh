# round-2 config sweep: Pippenger stream splits, cfg3 (4096 openings), cfg4 (BLS12-381), smoke
set -o pipefail
mkdir -p gpurun_out/r2/cfgs
for sp in 1 2 4; do
  timeout -k 10 300 python3 bench.py --fixed-bits 0 --split $sp --steps 10 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/cfgs/pip_split$sp.json 2> gpurun_out/r2/cfgs/pip_split$sp.err || { echo "pip split $sp failed"; tail -5 gpurun_out/r2/cfgs/pip_split$sp.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2/cfgs/pip_split$sp.json')); print('pip split $sp', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
timeout -k 10 400 python3 bench.py --workload cfg3 --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/cfgs/cfg3.json 2> gpurun_out/r2/cfgs/cfg3.err || { echo "cfg3 failed"; tail -5 gpurun_out/r2/cfgs/cfg3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2/cfgs/cfg3.json')); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'])"
timeout -k 10 400 python3 bench.py --workload cfg4 --no-latency --no-cpu-baseline > gpurun_out/r2/cfgs/cfg4.json 2> gpurun_out/r2/cfgs/cfg4.err || { echo "cfg4 failed"; tail -5 gpurun_out/r2/cfgs/cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2/cfgs/cfg4.json')); print('cfg4', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'], 'pip', round(d['secondary']['pippenger']['value']))"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/cfgs/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r2/cfgs/smoke.log; exit 1; }
tail -1 gpurun_out/r2/cfgs/smoke.log
