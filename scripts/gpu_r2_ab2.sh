# A/B: carry barrier after each column shift (asmcarry) vs baseline, table path c=17, interleaved
set -o pipefail
mkdir -p gpurun_out/r2/ab2
for rep in 1 2; do
  for v in base asmcarry; do
    if [ $v = asmcarry ]; then export KZGX_LIB=variants/asmcarry/libkzgx.so; else unset KZGX_LIB; fi
    timeout -k 10 300 python3 bench.py --no-pippenger --no-latency --no-cpu-baseline > gpurun_out/r2/ab2/${v}_$rep.json 2> gpurun_out/r2/ab2/${v}_$rep.err || { echo "$v failed"; tail -5 gpurun_out/r2/ab2/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r2/ab2/${v}_$rep.json')); print('$v', $rep, round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'], round(d['secondary']['valu_roofline']['peak_mixed_adds_per_s']/1e9,3))"
  done
done
