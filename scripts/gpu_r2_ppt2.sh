# interleaved A/B of the table path's decomposition on one box
set -o pipefail
mkdir -p gpurun_out/r2/ppt2
for rep in 1 2; do
for cfg in "16 1024" "11 1024" "22 2048" "11 2048"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --fixed-ppt $1 --batch $2 --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/ppt2/p$1_b$2_$rep.json 2> gpurun_out/r2/ppt2/p$1_b$2_$rep.err || { echo "ppt $1 b $2 failed"; tail -5 gpurun_out/r2/ppt2/p$1_b$2_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2/ppt2/p$1_b$2_$rep.json')); print('ppt $1 batch $2 rep $rep', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
done
