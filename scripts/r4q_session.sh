# round-4 session: single large table-less MSMs (the cfg5 rehearsal's 2^19
# partial ran 55 ms against 6.4 ms earlier); the lane-parallel inversion build
# (ab/libkzgx_inv4.so): its primitive latencies, default-table and parity
# tests on it, and single-call latency against the current build
I=ab/libkzgx_inv4.so
bash scripts/gpu.sh r4q py:big_msm.py && \
KZGX_LIB=$I bash scripts/gpu.sh r4q py:lat_micro.py tests:"default_table or parity or fixed" && \
bash scripts/lat_ab.sh r4q default KZGX_LIB=$I default KZGX_LIB=$I
