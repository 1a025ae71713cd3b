# round-4 final measurements: smoke, the default bench line and cfg3 / cfg4,
# the exact default command and a --serial run under rocprofv3 kernel stats
bash scripts/gpu.sh r4m smoke bench bench:--workload,cfg3 bench:--workload,cfg4 prof \
  prof:--serial,--steps,5,--no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup
