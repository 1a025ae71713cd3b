# round-4 session: GPU suite, single-call latency (Python and the C++ port of
# benchmark.cpp), default bench, traffic counter passes on the current kernel
Q=--serial,--steps,2,--warmup,1,--no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup
RD=TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum
bash scripts/gpu.sh r4i tests py:lat_floor.py && \
mkdir -p gpurun_out/r4i && timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4i/kzg_bench.txt 2>&1 && \
tail -3 gpurun_out/r4i/kzg_bench.txt && \
bash scripts/gpu.sh r4i bench pmc:$RD:$Q pmc:WRITE_SIZE:$Q pmc:$RD:$Q,--workload,cfg3 pmc:WRITE_SIZE:$Q,--workload,cfg3 pmc:$RD:$Q,--workload,cfg4 pmc:WRITE_SIZE:$Q,--workload,cfg4
