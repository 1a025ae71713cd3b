#!/bin/bash
# single-call latency under the Pippenger small-batch variants, one process
# each (the knobs are read once per process):
#   bash scripts/lat_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
for v in default KZGX_PIP_SEPARATE_MERGE=1 KZGX_PIP_SEPARATE_MERGE=1+KZGX_PIP_NO_FOLD_DIRECT=1 KZGX_PIP_KMIN=4; do
  envs=()
  [[ $v != default ]] && IFS=+ read -r -a envs <<< "$v"
  echo "== $v" >> "$OUT/lat_ab.txt"
  env "${envs[@]}" timeout -k 10 300 python3 -u scripts/lat_floor.py >> "$OUT/lat_ab.txt" 2>&1 || { tail -5 "$OUT/lat_ab.txt"; exit 1; }
done
cat "$OUT/lat_ab.txt"
