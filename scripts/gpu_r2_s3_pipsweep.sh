# Pippenger window / segment sweep on the current tree (BN254, 2048 per stream, 2 streams)
set -o pipefail
O=gpurun_out/r2/s3sw
mkdir -p $O
for cfg in "12 128" "13 128" "11 128" "12 256" "13 256"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --fixed-bits 0 --window-bits $1 --segment $2 --steps 10 --warmup 2 --no-cpu-baseline --no-latency > $O/pip_c$1_k$2.json 2> $O/pip_c$1_k$2.err || { echo "pip c$1 k$2 failed"; tail -5 $O/pip_c$1_k$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pip_c$1_k$2.json')); print('pip c=$1 K=$2', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
