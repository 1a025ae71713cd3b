# round-4 session: cooperative last fold levels and the two-level fold in the
# one-launch latency kernel (A/B against KZGX_NO_LAT_COOP and
# KZGX_LAT_THREADS=16384) and the one-workgroup quotient (KZGX_QWG_MIN=0),
# GPU suite, C++ benchmark port
bash scripts/gpu.sh r4l tests py:lat_micro.py && \
bash scripts/lat_ab.sh r4l default KZGX_NO_LAT_COOP=1 KZGX_LAT_THREADS=16384 KZGX_QWG_MIN=0 default KZGX_NO_LAT_COOP=1 KZGX_LAT_THREADS=16384 KZGX_QWG_MIN=0 && \
timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4l/kzg_bench.txt 2>&1 && \
tail -3 gpurun_out/r4l/kzg_bench.txt
