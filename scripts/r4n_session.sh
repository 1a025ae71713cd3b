# round-4 HBM traffic of k_fixed_accum on the final build: request-size and
# write counters in separate --pmc passes at the cfg2 / cfg3 / cfg4 shapes
# (scripts/pmc_traffic.py r4n 1 2 cfg2; 3 4 cfg3; 5 6 cfg4)
Q=--serial,--steps,2,--warmup,1,--no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup
RD=TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum
bash scripts/gpu.sh r4n pmc:$RD:$Q pmc:WRITE_SIZE:$Q pmc:$RD:$Q,--workload,cfg3 pmc:WRITE_SIZE:$Q,--workload,cfg3 \
  pmc:$RD:$Q,--workload,cfg4 pmc:WRITE_SIZE:$Q,--workload,cfg4
