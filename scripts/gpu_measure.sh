# memory query, c=17 / serial benches, PMC passes (each GPU step under its own limit)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python -c "import torch;p=torch.cuda.get_device_properties(0);print('total_memory',p.total_memory, torch.cuda.mem_get_info())" > gpurun_out/mem.txt 2>&1 || exit 1
cat gpurun_out/mem.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --serial > gpurun_out/bench_serial16.json 2> gpurun_out/bench_serial16.err || { tail -20 gpurun_out/bench_serial16.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_serial16.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['secondary'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --fixed-bits 17 > gpurun_out/bench_fb17.json 2> gpurun_out/bench_fb17.err || { tail -20 gpurun_out/bench_fb17.err; echo "fb17 failed"; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_fb17.json'));print(d['value'], d['config']['msm'], d['secondary'])" || true
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $pmc -d gpurun_out/pmc/$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --serial > gpurun_out/pmc_$tag.json 2> gpurun_out/pmc_$tag.err || { echo "pmc $tag failed"; tail -5 gpurun_out/pmc_$tag.err; exit 1; }
done
ls -R gpurun_out/pmc | head -30
