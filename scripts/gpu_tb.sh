# full GPU suite then bench variants
set -o pipefail
bash scripts/gpu_tests_all.sh || exit 1
VARIANTS_FILE=${VARIANTS_FILE:-scripts/variants4.txt} bash scripts/gpu_variants3.sh
