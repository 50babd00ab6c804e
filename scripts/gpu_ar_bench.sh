# xGMI IPC all-reduce latency, 2 and 4 ranks sharing the box's GPU (kernel overhead only).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 4; do
  DA_DIST_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench/allreduce_bench.py > gpurun_out/ar_bench_$n.json 2> gpurun_out/ar_bench_$n.err || { tail -20 gpurun_out/ar_bench_$n.err; exit 1; }
  cat gpurun_out/ar_bench_$n.json
done
