# round-4 session: single large table-less MSMs (2^14 ... 2^20 + 1 points);
# the Pippenger small-batch fold's whole-wavefront conversion (parity tests,
# table-off single-call latency)
bash scripts/gpu.sh r4r py:big_msm.py && \
bash scripts/gpu.sh r4r_t tests:"parity or default_table or workspace" && \
bash scripts/lat_ab.sh r4r_l LAT_NO_DEFAULT_TABLE=1 default
