# round-4 last lines on the final build: the default bench and cfg3
bash scripts/gpu.sh r4w bench bench:--workload,cfg3,--no-cpu-baseline
