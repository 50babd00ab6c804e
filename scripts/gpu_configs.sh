# BASELINE configs and rehearsals through bench.py on the box's one GPU: bash scripts/gpu_configs.sh CASE
#   c3        Llama-3-8B summarizer + QA, PDF ingest (gateway PDF extraction in the timed ingest path)
#   c4        BGE-large embedder, 1.25M-chunk shard (= 10M sharded 8-way), Phi-3-mini QA
#   c4f16     the same with the embedder in fp16 (BASELINE config 4 "BGE-large fp16 embedder")
#   llama70b  Llama-3-70B QA on one GPU (TP=1), BGE-large
#   rank2     2 ranks sharing the GPU (gloo collectives): the multi-rank bench path
#   tp2       Phi-3-mini TP=2 + IVFFlat, 2 ranks sharing the GPU (xGMI IPC all-reduce kernel, gloo)
#   c5        BASELINE config 5 layout: Llama-3-70B TP=8 + fp8 encoder + IVFFlat, 8 ranks sharing the GPU
#   r2/r4/r8  the driver's N > 1 bench path rehearsed with 2 / 4 / 8 ranks sharing the GPU (gloo; small batch):
#             every block (rccl_search, tp_decode, tp_decode_70b at 8, xgmi_allreduce, serving_search)
#   c4full    BASELINE config 4 at its real total size: 8 ranks x 1.25M rows (10M), BGE-large fp16, the
#             rccl-form sharded search in the QA step; then recall vs one exact 10M-row index
#   index     vector index microbenchmarks (flat / IVFFlat, up to 100M x 1024 rows)
#   xgmi      IPC all-reduce GPU tests (2 ranks sharing the GPU)
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 3; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.err; cat gpurun_out/$name.json
  return $rc
}
case ${1:-c4} in
  c3) run c3 900 python bench.py --llm llama3-8b --pdf-ingest ;;
  c4) run c4 600 python bench.py --enc bge-large --index-rows 1250000 --latency-reps 3 --ingest-docs 32 ;;
  c4f16) run c4f16 600 python bench.py --enc bge-large --enc-dtype fp16 --index-rows 1250000 --latency-reps 3 \
           --ingest-docs 32 ;;
  llama70b) run llama70b 1200 python bench.py --llm llama3-70b --enc bge-large --batch 16 --steps 2 --warmup 1 \
              --latency-reps 2 --ingest-docs 4 --ingest-batches 1 ;;
  rank2) DA_DIST_BACKEND=gloo run rank2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
           --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 16 \
           --latency-reps 2 --ingest-docs 4 --ingest-batches 1 ;;
  tp2) DA_DIST_BACKEND=gloo run tp2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
         --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --tp 2 --index-kind ivfflat --steps 1 \
         --warmup 1 --batch 8 --latency-reps 1 --ingest-docs 0 ;;
  c5) DA_DIST_BACKEND=gloo run c5 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --llm llama3-70b --tp 8 --enc bge-large \
        --enc-dtype fp8 --index-kind ivfflat --batch 2 --steps 1 --warmup 1 --latency-reps 1 --ingest-docs 0 \
        --max-new 8 --breakdown 0 ;;  # gloo TP all-reduces through the host: a path check, not a perf number
  r2) DA_DIST_BACKEND=gloo run r2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 \
        --latency-reps 2 --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 ;;
  r4) DA_DIST_BACKEND=gloo run r4 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29540 bench.py --gpus 4 --steps 1 --warmup 1 --batch 4 \
        --latency-reps 1 --ingest-docs 2 --ingest-batches 1 --ingest-latency-reps 1 --max-new 8 --breakdown 0 ;;
  r8) DA_DIST_BACKEND=gloo run r8 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 8 --steps 1 --warmup 1 --batch 4 \
        --latency-reps 1 --ingest-docs 2 --ingest-batches 1 --ingest-latency-reps 1 --max-new 8 \
        --tp70b-batches 1,2 --breakdown 0 ;;
  c4full) DA_DIST_BACKEND=gloo run c4full 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --enc bge-large --enc-dtype fp16 \
            --index-rows 1250000 --batch 4 --steps 2 --warmup 1 --latency-reps 2 --ingest-docs 0 --max-new 8 \
            --breakdown 0 --tp70b off --search rccl \
          && DA_DIST_BACKEND=gloo run c4recall 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port 29539 bench/sharded_recall.py --rows 1250000 --dim 1024 \
            --queries 64 ;;
  index) run index_flat 600 python bench/index_bench.py --kind flat --rows 10000000 --dim 1024 \
           && run index_ivf 900 python bench/index_bench.py --kind ivfflat --rows 10000000 --dim 1024 --lists 4096 \
              --probes 4,16,64 ;;
  xgmi) timeout -k 10 300 python -u -m pytest tests/test_xgmi_allreduce_gpu.py -x -v -p no:cacheprovider --timeout 240 \
          --timeout-method thread > gpurun_out/t_ar.log 2>&1; rc=$?; tail -20 gpurun_out/t_ar.log; exit $rc ;;
  *) echo "unknown case $1"; exit 2 ;;
esac
