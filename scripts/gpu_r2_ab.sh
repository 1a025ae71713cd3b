# A/B on one box: 80-B (l29) vs 64-B packed table at c=16, and packed c=17, interleaved twice
set -o pipefail
mkdir -p gpurun_out/r2/ab
for rep in 1 2; do
  for v in l29_16 packed_16 packed_17; do
    if [ $v = l29_16 ]; then export KZGX_LIB=variants/l29/libkzgx.so; else unset KZGX_LIB; fi
    c=${v##*_}
    timeout -k 10 300 python3 bench.py --fixed-bits $c --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/ab/${v}_$rep.json 2> gpurun_out/r2/ab/${v}_$rep.err || { echo "$v failed"; tail -5 gpurun_out/r2/ab/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r2/ab/${v}_$rep.json')); print('$v', $rep, round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
  done
done
