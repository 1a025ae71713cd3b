# A/B: accumulation occupancy variants and window widths (bench cfg2, no CPU baseline)
set -o pipefail
for v in ${VARIANTS:-w3 w4}; do
  KZGX_LIB=$PWD/variants/libkzgx_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${EXTRA:-} > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || { echo "$v failed"; tail gpurun_out/var_$v.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/var_$v.json'));print('$v',round(j['value']),j['parity'],{k:round(v,2) for k,v in j['secondary']['kernel_ms_per_step'].items()})"
done
for c in ${WINDOWS:-11 13}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --window-bits $c > gpurun_out/var_c$c.json 2>gpurun_out/var_c$c.err || { echo "c$c failed"; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/var_c$c.json'));print('c$c',round(j['value']),j['parity'],{k:round(v,2) for k,v in j['secondary']['kernel_ms_per_step'].items()})"
done
