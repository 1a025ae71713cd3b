# tests -> bench -> rocprofv3 kernel stats, each GPU step under its own limit
set -o pipefail
bash scripts/gpu_test_bench.sh || exit 1
bash scripts/gpu_prof.sh || exit 1
