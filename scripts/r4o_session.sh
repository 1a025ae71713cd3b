# round-4 A/B: points per thread of the automatic batched table path (the
# default table's batches) from 1024 MSMs, 16 against 22 (BN254) / 65 (BLS12-381)
L=kzg-commitments_amd/libkzgx.so
bash scripts/gpu_ab.sh r4o_cfg2 $L $L+KZGX_PPT_AUTO_BIG=22 --no-latency,--no-table-curve,--no-cpu-baseline,--no-setup,--steps,5 2 && \
bash scripts/gpu_ab.sh r4o_cfg4 $L $L+KZGX_PPT_AUTO_BIG=65 --workload,cfg4,--no-latency,--no-table-curve,--no-cpu-baseline,--no-setup,--steps,5 2
