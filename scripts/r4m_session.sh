# round-4 final measurements: GPU suite, smoke, the default bench line and
# the cfg3 / cfg4 lines
bash scripts/gpu.sh r4m tests smoke bench bench:--workload,cfg3 bench:--workload,cfg4
