#!/bin/bash
# Builds scripts/mb/merge_bN.co, the inlined k_msm_merge<BN254G1> alone
# (scripts/repro_merge_mod.hip) with -mllvm -opt-bisect-limit=N (LLVM runs
# optional passes 1..N and skips the rest), for each N given, plus the
# driver scripts/mb/repro_merge_fast.  On the GPU:
#   for c in scripts/mb/merge_b*.co; do REPRO_CO=$c scripts/mb/repro_merge_fast | head -1; done
# names the first pass after which the inlined merge disagrees with the
# expected sums.  Pass numbers: build with -opt-bisect-limit=-1 and read stderr.
#
#   bash scripts/merge_bisect.sh 2000 2500 ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p scripts/mb
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DREPRO_FAST -o scripts/mb/repro_merge_fast \
  scripts/repro_merge.hip > /tmp/merge_bisect_driver.log 2>&1 &
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output \
    -mllvm -opt-bisect-limit="$n" -o "scripts/mb/merge_b$n.co" scripts/repro_merge_mod.hip \
    > "/tmp/merge_bisect_$n.log" 2>&1 &
  while [ "$(jobs -r | wc -l)" -ge 8 ]; do sleep 1; done
done
wait
for n in "$@"; do
  [ -s "scripts/mb/merge_b$n.co" ] && echo "built $n" || echo "FAILED $n (/tmp/merge_bisect_$n.log)"
done
