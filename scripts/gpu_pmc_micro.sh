set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
BIN=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/p1 -o p1 --output-format csv -- ./scripts/mb/$BIN > $OUT/p1.log 2>&1
echo "exit $?"
