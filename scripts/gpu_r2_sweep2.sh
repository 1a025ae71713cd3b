# Pippenger window sweep (c = 11, 12, 13) and BLS12-381 table layout A/B (96-B packed vs 112-B radix-2^29)
set -o pipefail
mkdir -p gpurun_out/r2/sw2
for c in 11 13 12; do
  timeout -k 10 300 python3 bench.py --fixed-bits 0 --window-bits $c --steps 10 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/r2/sw2/pip_c$c.json 2> gpurun_out/r2/sw2/pip_c$c.err || { echo "pip c$c failed"; tail -5 gpurun_out/r2/sw2/pip_c$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2/sw2/pip_c$c.json')); print('pip c$c', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
for rep in 1 2; do
for v in packed l29; do
  if [ $v = l29 ]; then export KZGX_LIB=variants/l29/libkzgx.so; else unset KZGX_LIB; fi
  timeout -k 10 400 python3 bench.py --workload cfg4 --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/sw2/bls_$v$rep.json 2> gpurun_out/r2/sw2/bls_$v$rep.err || { echo "bls $v failed"; tail -5 gpurun_out/r2/sw2/bls_$v$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2/sw2/bls_$v$rep.json')); print('bls $v', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'])"
done
done
