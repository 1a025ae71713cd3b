# round-4 closing: the Q64 and 8-wavefront quotient defaults -- GPU suite,
# smoke, single-call latency, C++ benchmark port
bash scripts/gpu.sh r4v tests smoke py:lat_floor.py && \
timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4v/kzg_bench.txt 2>&1 && \
tail -2 gpurun_out/r4v/kzg_bench.txt
