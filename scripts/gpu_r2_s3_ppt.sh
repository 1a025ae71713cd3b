# cfg3 points-per-thread A/B (16: 5 wavefronts per MSM, 6.7 residencies; 22: 3 per MSM, 4 residencies),
# (BLS12-381 at 3 wavefronts per SIMD was built and rejected at compile time: 111 VGPRs spilled)
set -o pipefail
O=gpurun_out/r2/s3w3
mkdir -p $O
for rep in 1 2; do
for p in 16 22; do
  timeout -k 10 400 python3 bench.py --workload cfg3 --fixed-ppt $p --no-pippenger --no-latency --no-cpu-baseline > $O/cfg3_p${p}_$rep.json 2> $O/cfg3_p${p}_$rep.err || { echo "cfg3 $p failed"; tail -5 $O/cfg3_p${p}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg3_p${p}_$rep.json')); print('cfg3 ppt=$p', round(d['value']), round(d['ms_per_step'],3), d['parity']['ok'])"
done
done
timeout -k 10 400 python3 bench.py --workload cfg4 --no-latency --no-cpu-baseline > $O/cfg4_default.json 2> $O/cfg4_default.err || { echo "cfg4 failed"; tail -5 $O/cfg4_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg4_default.json')); print('cfg4 default', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'], 'pip', round(d['secondary']['pippenger']['value']))"
