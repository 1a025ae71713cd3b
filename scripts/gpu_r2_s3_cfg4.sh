# cfg4 (BLS12-381, table c = 16, 2 waves per SIMD = 2048 resident wavefronts): batch x points-per-thread
# shapes that fill whole residencies, interleaved with the default (B = 1024, 16 points per thread)
set -o pipefail
O=gpurun_out/r2/s3cfg4
mkdir -p $O
for rep in 1 2; do
for shape in "1024 16" "1024 33" "2048 33" "2048 65"; do
  set -- $shape
  timeout -k 10 400 python3 bench.py --workload cfg4 --batch $1 --fixed-ppt $2 --no-pippenger --no-latency --no-cpu-baseline > $O/cfg4_b$1_p$2_$rep.json 2> $O/cfg4_b$1_p$2_$rep.err || { echo "cfg4 $shape failed"; tail -5 $O/cfg4_b$1_p$2_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg4_b$1_p$2_$rep.json')); print('cfg4 B=$1 ppt=$2', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'], round(d['secondary']['valu_roofline']['frac'],3))"
done
done
