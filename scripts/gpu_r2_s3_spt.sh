# Pippenger count/scatter block size A/B (scalars per thread 2 = default, 3, 4), interleaved;
# each variant first runs the Pippenger parity tests
set -o pipefail
O=gpurun_out/r2/s3spt
mkdir -p $O
for v in 3 4; do
  KZGX_LIB=variants/spt$v/libkzgx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pippenger_buckets.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_spt$v.log 2>&1; rc=$?
  tail -1 $O/tests_spt$v.log
  [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/tests_spt$v.log | head -20; exit $rc; }
done
for rep in 1 2; do
for v in 2 3 4; do
  if [ $v = 2 ]; then unset KZGX_LIB; else export KZGX_LIB=variants/spt$v/libkzgx.so; fi
  timeout -k 10 300 python3 bench.py --fixed-bits 0 --steps 10 --warmup 2 --no-cpu-baseline --no-latency > $O/pip_spt${v}_$rep.json 2> $O/pip_spt${v}_$rep.err || { echo "spt $v failed"; tail -5 $O/pip_spt${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pip_spt${v}_$rep.json')); print('pip spt=$v', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
done
