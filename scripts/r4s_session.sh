# round-4 session: the Pippenger small-batch fold's whole-wavefront
# conversion (parity tests, table-off single-call latency); cfg5 on the
# table-less path at one rank and at two ranks on one device (the 2-rank
# rehearsal's partial MSM read 55 ms where one 2^19-point MSM takes 2.8 ms)
bash scripts/gpu.sh r4s_t tests:"parity or default_table or workspace" && \
bash scripts/lat_ab.sh r4s_l LAT_NO_DEFAULT_TABLE=1 default && \
bash scripts/gpu.sh r4s_b bench:--workload,cfg5,--steps,5,--warmup,1,--table-gb,60,--no-cpu-baseline && \
KZGX_BENCH_ONE_DEVICE=1 KZGX_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --workload cfg5 --steps 5 \
  --warmup 1 --table-gb 60 --no-cpu-baseline > gpurun_out/r4s_b/cfg5_2rank.json 2> gpurun_out/r4s_b/cfg5_2rank.err && \
tail -c 600 gpurun_out/r4s_b/cfg5_2rank.json
