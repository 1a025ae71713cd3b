#!/bin/bash
# single-call latency (scripts/lat_floor.py) under environment variants, one
# process each (the knobs are read once per process):
#   bash scripts/lat_ab.sh TAG [VARIANT ...]   (VARIANT: default or A=1+B=2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
TAG=$1
shift
VARIANTS=("$@")
[[ ${#VARIANTS[@]} -eq 0 ]] && VARIANTS=(default KZGX_PIP_SEPARATE_MERGE=1 KZGX_PIP_SEPARATE_MERGE=1+KZGX_PIP_NO_FOLD_DIRECT=1 KZGX_PIP_KMIN=4)
for v in "${VARIANTS[@]}"; do
  envs=()
  [[ $v != default ]] && IFS=+ read -r -a envs <<< "$v"
  echo "== $v" >> "$OUT/lat_ab.txt"
  env "${envs[@]}" timeout -k 10 300 python3 -u scripts/lat_floor.py >> "$OUT/lat_ab.txt" 2>&1 || { tail -5 "$OUT/lat_ab.txt"; exit 1; }
done
cat "$OUT/lat_ab.txt"
