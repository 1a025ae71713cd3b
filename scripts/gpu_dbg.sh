set -o pipefail
mkdir -p gpurun_out/r2
for v in seq nopf; do
  if [ $v = main ]; then unset KZGX_LIB; else export KZGX_LIB=variants/$v/libkzgx.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "test_msm_matches_naive or window_and_segment" > gpurun_out/r2/dbg_$v.log 2>&1
  echo "== $v"; grep -E "PASSED|FAILED" gpurun_out/r2/dbg_$v.log | sed 's/tests\/test_gpu_parity.py:://' | awk '{print $1, $2}' | grep -c PASSED
  grep -E "FAILED" gpurun_out/r2/dbg_$v.log | head -5
done
exit 0
