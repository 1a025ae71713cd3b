# table path work decomposition: points per thread and batch size (default c=17)
set -o pipefail
mkdir -p gpurun_out/r2/ppt
for cfg in "16 1024" "22 1024" "11 1024" "32 1024" "22 2048" "16 2048"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --fixed-ppt $1 --batch $2 --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/ppt/p$1_b$2.json 2> gpurun_out/r2/ppt/p$1_b$2.err || { echo "ppt $1 b $2 failed"; tail -5 gpurun_out/r2/ppt/p$1_b$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2/ppt/p$1_b$2.json')); print('ppt $1 batch $2', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'], {k: round(v,3) for k,v in d['secondary']['kernel_ms_per_step'].items() if v})"
done
