# GPU parity tests then the default bench; each GPU step under its own limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "^E |FAILED" gpurun_out/tests.log | head -20; exit 1; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
