# current-tree refresh of the verify-half timings (both curves) and the --benchmark-common sweep
set -o pipefail
O=gpurun_out/r2/s3v
mkdir -p $O
for c in BN254 BLS12381; do
  timeout -k 10 300 python3 scripts/bench_verify.py --curve $c > $O/verify_$c.json 2> $O/verify_$c.err || { echo "verify $c failed"; tail -10 $O/verify_$c.err; exit 1; }
  head -c 600 $O/verify_$c.json; echo
done
timeout -k 10 600 python3 bench.py --workload common > $O/common.json 2> $O/common.err || { echo "common failed"; tail -20 $O/common.err; exit 1; }
grep common: $O/common.err | tail -12
