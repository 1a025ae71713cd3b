set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro_madd > gpurun_out/r3_micro_madd.txt 2>&1 && \
KZGX_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 1 --fixed-bits 12 --no-cpu-baseline --no-pippenger --no-latency > gpurun_out/r3_rccl_cfg2.json 2> gpurun_out/r3_rccl_cfg2.err
echo "exit $?"
tail -3 gpurun_out/r3_rccl_cfg2.err
