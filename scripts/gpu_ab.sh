#!/bin/bash
# A/B of two builds of libkzgx.so on one box, interleaved:
#   bash scripts/gpu_ab.sh TAG LIB_A LIB_B "bench args (commas)" [rounds]
# LIB_A / LIB_B: a libkzgx.so path, optionally followed by environment
# settings for that side: path+VAR=value+VAR2=value
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1; A=$2; B=$3; ARGS=${4//,/ }; R=${5:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in A B; do
    spec=$A; [[ $v == B ]] && spec=$B
    IFS=+ read -r lib envs <<< "$spec"
    envargs=()
    [[ -n "$envs" ]] && IFS=+ read -r -a envargs <<< "$envs"
    env KZGX_LIB="$lib" "${envargs[@]}" timeout -k 10 500 python -u bench.py $ARGS > "$OUT/${v}_$r.json" \
      2> "$OUT/${v}_$r.err" || { tail -20 "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, round(d['value']), d['parity'])"
  done
done
