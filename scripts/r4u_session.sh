# round-4 A/B: <= 64 wavefront partials for small single MSMs (KZGX_LAT_Q64=1)
# and the one-workgroup quotient at 8 wavefronts (KZGX_QWG_WAVES=8); the
# default-table / quotient tests under both knobs
KZGX_LAT_Q64=1 KZGX_QWG_WAVES=8 bash scripts/gpu.sh r4u_t tests:default_table && \
bash scripts/lat_ab.sh r4u default KZGX_LAT_Q64=1 KZGX_QWG_WAVES=8 default KZGX_LAT_Q64=1 KZGX_QWG_WAVES=8
