#!/bin/bash
# N-rank rehearsal of bench.py's self-launcher on a one-GPU box: every rank
# on device 0 (KZGX_BENCH_ONE_DEVICE=1); RCCL refuses two ranks on one
# device ("Duplicate GPU detected", profiles/r03_rccl_one_device.txt), so the
# timing reductions and the cfg5 all-gather use gloo here.
#   bash scripts/gpu_rehearse.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
export KZGX_BENCH_ONE_DEVICE=1 KZGX_DIST_BACKEND=gloo
timeout -k 10 500 python -u bench.py --gpus 2 --steps 5 --warmup 1 --fixed-bits 12 --no-cpu-baseline --no-pippenger \
  --no-latency --no-table-curve > "$OUT/cfg2_2rank.json" 2> "$OUT/cfg2_2rank.err" || { tail -20 "$OUT/cfg2_2rank.err"; exit 1; }
tail -c 300 "$OUT/cfg2_2rank.json"
timeout -k 10 500 python -u bench.py --gpus 2 --workload cfg5 --steps 5 --warmup 1 --table-gb 60 --no-cpu-baseline \
  > "$OUT/cfg5_2rank.json" 2> "$OUT/cfg5_2rank.err" || { tail -20 "$OUT/cfg5_2rank.err"; exit 1; }
tail -c 300 "$OUT/cfg5_2rank.json"
# strong scaling: a fixed total batch split over the ranks
timeout -k 10 500 python -u bench.py --gpus 2 --scaling strong --global-batch 4096 --steps 5 --warmup 1 --fixed-bits 12 \
  --no-cpu-baseline --no-pippenger --no-latency --no-table-curve > "$OUT/cfg2_2rank_strong.json" \
  2> "$OUT/cfg2_2rank_strong.err" || { tail -20 "$OUT/cfg2_2rank_strong.err"; exit 1; }
tail -c 300 "$OUT/cfg2_2rank_strong.json"
