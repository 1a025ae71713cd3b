# flat kernel with two lookups in flight: its tests, then cfg5 A/B: T = 1x / 2x the resident lanes, point-strided
set -o pipefail
O=gpurun_out/r2/s3flat2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_fixed.log 2>&1; rc=$?
tail -3 $O/tests_fixed.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/tests_fixed.log | head -30; exit $rc; }
for rep in 1 2; do
for v in t1 t2 strided; do
  unset KZGX_NO_FIXED_FLAT KZGX_FLAT_TMULT
  if [ $v = strided ]; then export KZGX_NO_FIXED_FLAT=1; fi
  if [ $v = t2 ]; then export KZGX_FLAT_TMULT=2; fi
  timeout -k 10 300 python3 bench.py --workload cfg5 --no-cpu-baseline > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.err || { echo "cfg5 $v failed"; tail -5 $O/cfg5_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_${v}_$rep.json')); print('cfg5 $v', round(d['value'],1), round(d['ms_per_step'],3), d['parity']['ok'], round(d['secondary']['valu_roofline']['frac'],3))"
done
done
