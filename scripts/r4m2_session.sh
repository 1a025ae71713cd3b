# round-4 final profiles: the exact default command and a --serial run under
# rocprofv3 kernel stats
bash scripts/gpu.sh r4m2 prof prof:--serial,--steps,5,--no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup
