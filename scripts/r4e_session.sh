bash scripts/gpu.sh r4e tests py:lat_floor.py && \
bash scripts/gpu_ab.sh r4e_pip kzg-commitments_amd/libkzgx.so+KZGX_PIP_DIRECT_SCATTER=1 kzg-commitments_amd/libkzgx.so --fixed-bits,0,--no-latency,--no-cpu-baseline,--no-setup,--no-table-curve 2 && \
bash scripts/gpu_ab.sh r4e_sgpr kzg-commitments_amd/libkzgx.so variants/plsgpr/libkzgx.so --no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup 2 && \
bash scripts/gpu_rehearse.sh r4e_rh && \
bash scripts/gpu.sh r4e prof:--fixed-bits,0,--no-latency,--no-cpu-baseline,--no-setup,--no-table-curve,--serial,--steps,4
