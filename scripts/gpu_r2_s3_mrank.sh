# rehearse bench.py's N = 2 control flow on a one-GPU box (two ranks on device 0 over gloo):
# cfg2 with a small table, cfg5 with a table over each rank's 2^19-point shard (flat kernel path)
set -o pipefail
O=gpurun_out/r2/s3mrank
mkdir -p $O
export KZGX_BENCH_ONE_DEVICE=1 KZGX_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --fixed-bits 12 --no-latency > $O/cfg2.json 2> $O/cfg2.err || { echo "2-rank cfg2 failed"; tail -20 $O/cfg2.err; exit 1; }
cut -c1-400 $O/cfg2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload cfg5 --steps 3 --warmup 1 --table-gb 80 > $O/cfg5.json 2> $O/cfg5.err || { echo "2-rank cfg5 failed"; tail -20 $O/cfg5.err; exit 1; }
cut -c1-1200 $O/cfg5.json
