# Pippenger bucket fold A/B: the one-wavefront fold + thread-per-MSM finish
# (KZGX_PIP_WAVE_FOLD=1) against the workgroup fold, at several batch sizes
set -o pipefail
O=gpurun_out/r2/s3fold
mkdir -p $O
for B in 2048 512 128; do
for v in wg wave; do
  if [ $v = wave ]; then export KZGX_PIP_WAVE_FOLD=1; else unset KZGX_PIP_WAVE_FOLD; fi
  timeout -k 10 300 python3 bench.py --fixed-bits 0 --batch $B --steps 10 --warmup 2 --no-cpu-baseline --no-latency > $O/pip_${v}_$B.json 2> $O/pip_${v}_$B.err || { echo "pip $v $B failed"; tail -5 $O/pip_${v}_$B.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pip_${v}_$B.json')); print('pip $v B=$B', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
done
