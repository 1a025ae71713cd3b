# round-4 session: cooperative last fold levels in the one-launch latency
# kernel (A/B against KZGX_NO_LAT_COOP), GPU suite, C++ benchmark port
bash scripts/gpu.sh r4l tests py:lat_micro.py && \
bash scripts/lat_ab.sh r4l default KZGX_NO_LAT_COOP=1 default KZGX_NO_LAT_COOP=1 && \
timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4l/kzg_bench.txt 2>&1 && \
tail -3 gpurun_out/r4l/kzg_bench.txt
