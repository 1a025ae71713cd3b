# A/B: sub-batch stream split of the cfg2 bench (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
for s in ${SPLITS:-1 2 4}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --split $s ${EXTRA:-} > gpurun_out/split_$s.json 2>gpurun_out/split_$s.err || { echo "split $s failed"; tail gpurun_out/split_$s.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/split_$s.json'));print('split $s',round(j['value']),j['parity'],{k:round(v,2) for k,v in j['secondary']['kernel_ms_per_step'].items()})"
done
