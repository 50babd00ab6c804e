# Rehearse the multi-rank bench path (2 ranks sharing the box's one GPU, gloo for the collectives).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
DA_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 16 --latency-reps 2 --ingest-docs 4 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?
echo "bench2 rc=$rc"; tail -5 gpurun_out/bench2.err; cat gpurun_out/bench2.json
exit $rc
