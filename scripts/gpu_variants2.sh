# bench variants; each GPU step under its own limit; args: list of "name|bench args"
set -o pipefail
mkdir -p gpurun_out/var
while IFS= read -r line; do
  [ -z "$line" ] && continue
  name="${line%%|*}"; args="${line#*|}"
  timeout -k 10 600 python bench.py --no-cpu-baseline $args > gpurun_out/var/$name.json 2> gpurun_out/var/$name.err || { echo "bench $name failed"; tail -20 gpurun_out/var/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var/$name.json'));print('$name', round(d['value']), d['config'].get('msm'), {k:round(v,3) for k,v in d['secondary']['kernel_ms_per_step'].items() if v})"
done < "${VARIANTS_FILE:-scripts/variants.txt}"
