# bench variants with optional alternative library builds; lines "name|lib or -|bench args"
set -o pipefail
mkdir -p gpurun_out/var
while IFS= read -r line; do
  [ -z "$line" ] && continue
  name="${line%%|*}"; rest="${line#*|}"; lib="${rest%%|*}"; args="${rest#*|}"
  if [ "$lib" = "-" ]; then unset KZGX_LIB; else export KZGX_LIB=$lib; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/var/$name.json 2> gpurun_out/var/$name.err || { echo "bench $name failed"; tail -20 gpurun_out/var/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var/$name.json'));print('$name', round(d['value']), d['config'].get('msm'), {k:round(v,3) for k,v in d['secondary']['kernel_ms_per_step'].items() if v})"
done < "${VARIANTS_FILE:-scripts/variants3.txt}"
