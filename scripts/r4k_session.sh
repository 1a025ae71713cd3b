# round-4 session: the budget-chosen default table (BN254 c = 11, BLS12-381
# c = 10) and the scalar-ALU inversion of single-lane tails: GPU suite,
# primitive latencies, single-call latency, C++ benchmark port, cfg2 and cfg4
bash scripts/gpu.sh r4k tests py:lat_micro.py py:lat_floor.py && \
mkdir -p gpurun_out/r4k && timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4k/kzg_bench.txt 2>&1 && \
tail -3 gpurun_out/r4k/kzg_bench.txt && \
bash scripts/gpu.sh r4k bench bench:--workload,cfg4
