# round-4 session: GPU suite, single-call latency, Pippenger A/Bs (direct
# scatter + separate merge vs block-major + fused; block-major + separate
# merge), SGPR modulus limbs A/B on cfg2, 2-rank rehearsal, serial profile
P=--fixed-bits,0,--no-latency,--no-cpu-baseline,--no-setup,--no-table-curve
L=kzg-commitments_amd/libkzgx.so
bash scripts/gpu.sh r4e tests py:lat_floor.py && \
bash scripts/gpu_ab.sh r4e_pip $L+KZGX_PIP_DIRECT_SCATTER=1+KZGX_PIP_SEPARATE_MERGE=1 $L $P 2 && \
bash scripts/gpu_ab.sh r4e_pip2 $L+KZGX_PIP_SEPARATE_MERGE=1 $L $P 1 && \
bash scripts/gpu_ab.sh r4e_sgpr $L variants/plsgpr/libkzgx.so --no-pippenger,--no-table-curve,--no-latency,--no-cpu-baseline,--no-setup 2 && \
bash scripts/gpu_rehearse.sh r4e_rh && \
bash scripts/gpu.sh r4e prof:$P,--serial,--steps,4
