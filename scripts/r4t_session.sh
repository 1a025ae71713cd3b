# round-4 final session on the committed build: GPU suite, smoke, the C++
# port of the reference benchmark, the default bench line
bash scripts/gpu.sh r4t tests smoke && \
timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4t/kzg_bench.txt 2>&1 && \
tail -2 gpurun_out/r4t/kzg_bench.txt && \
bash scripts/gpu.sh r4t_b bench
