# round-4 closing session on the final build: GPU suite, smoke, the 2-rank
# self-launch rehearsal (weak, strong, cfg5; gloo on one device) and cfg4
bash scripts/gpu.sh r4p tests smoke && \
bash scripts/gpu_rehearse.sh r4p && \
bash scripts/gpu.sh r4p bench:--workload,cfg4,--no-cpu-baseline
