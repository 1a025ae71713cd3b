# rehearse bench.py's N = 2 control flow on a one-GPU box: two ranks on device 0 over gloo, small table
set -o pipefail
mkdir -p gpurun_out/r2
export KZGX_BENCH_ONE_DEVICE=1 KZGX_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --fixed-bits 12 --no-latency > gpurun_out/r2/mrank.json 2> gpurun_out/r2/mrank.err || { echo "2-rank bench failed"; tail -20 gpurun_out/r2/mrank.err; exit 1; }
cat gpurun_out/r2/mrank.json | cut -c1-700
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload cfg5 --steps 3 --warmup 1 --fixed-bits 0 > gpurun_out/r2/mrank5.json 2> gpurun_out/r2/mrank5.err || { echo "2-rank cfg5 failed"; tail -20 gpurun_out/r2/mrank5.err; exit 1; }
cat gpurun_out/r2/mrank5.json | cut -c1-700
