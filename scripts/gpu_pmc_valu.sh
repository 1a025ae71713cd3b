# VALU counters for the accum kernel (one PMC pass) + C++ facade test
set -o pipefail
mkdir -p gpurun_out/pmc_valu
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_valu/SQ -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --serial > gpurun_out/pmc_valu.json 2> gpurun_out/pmc_valu.err || { echo "pmc failed"; tail -5 gpurun_out/pmc_valu.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_cpp_api.py -x -q --timeout 250 --timeout-method thread > gpurun_out/cpp.log 2>&1; rc=$?
tail -3 gpurun_out/cpp.log; exit $rc
