# A/B: default bench (cfg2) with the point-strided k_fixed_accum vs its two-lookups-in-flight variant
# (variants/pf2, -DKZGX_FIXED_PREFETCH2), interleaved; then the 8-GPU cfg5 shard size (2^17 points,
# c = 10) flat vs point-strided
set -o pipefail
O=gpurun_out/r2/s3pf2
mkdir -p $O
for rep in 1 2; do
for v in base pf2; do
  if [ $v = pf2 ]; then export KZGX_LIB=variants/pf2/libkzgx.so; else unset KZGX_LIB; fi
  timeout -k 10 300 python3 bench.py --no-pippenger --no-latency --no-cpu-baseline > $O/cfg2_${v}_$rep.json 2> $O/cfg2_${v}_$rep.err || { echo "cfg2 $v failed"; tail -5 $O/cfg2_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg2_${v}_$rep.json')); print('cfg2 $v', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'], round(d['secondary']['valu_roofline']['frac'],3))"
done
done
unset KZGX_LIB
for v in flat strided; do
  if [ $v = strided ]; then export KZGX_NO_FIXED_FLAT=1; else unset KZGX_NO_FIXED_FLAT; fi
  timeout -k 10 300 python3 scripts/flat_small.py 131073 10 > $O/shard8_$v.json 2> $O/shard8_$v.err || { echo "shard8 $v failed"; tail -5 $O/shard8_$v.err; exit 1; }
  cat $O/shard8_$v.json
done
