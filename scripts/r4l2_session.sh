# round-4 session: the one-workgroup quotient at 4 wavefronts (one per SIMD)
# against the chip-wide / one-wavefront kernels (KZGX_QWG_MIN=0), latency
# threads back to 2^14 per MSM; default-table and quotient tests
bash scripts/gpu.sh r4l2 tests:default_table && \
bash scripts/lat_ab.sh r4l2 default KZGX_QWG_MIN=0 default KZGX_QWG_MIN=0 && \
timeout -k 10 300 ./kzg-commitments_amd/tools/kzg_bench > gpurun_out/r4l2/kzg_bench.txt 2>&1 && \
tail -3 gpurun_out/r4l2/kzg_bench.txt
