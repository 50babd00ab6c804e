# BASELINE configs 4 and 5 through bench.py on the box's one GPU:
#  4: BGE-large embedder, 1.25M-chunk shard (= 10M sharded 8-way), Phi-3-mini QA, 1 rank
#  TP rehearsal: phi3-mini TP=2 (2 ranks sharing the GPU, gloo + the xGMI IPC all-reduce kernel)
#  5: Llama-3-70B TP=8 + fp8 encoder GEMMs + IVFFlat index, 8 ranks sharing the GPU (correctness
#     rehearsal of the 8-GPU layout; gloo carries the large prefill all-reduces, so not a perf number:
#     the warmup QA step completes, the timed step outlasts gpurun's 180-s silence limit —
#     profiles/config5_llama70b_tp8_rehearsal_8rank_1gpu.log). RUN_C5=1 to include it.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
if [ "${SKIP_C4:-0}" != 1 ]; then
timeout -k 10 600 python bench.py --enc bge-large --index-rows 1250000 --latency-reps 3 --ingest-docs 32 > gpurun_out/c4.json 2> gpurun_out/c4.err
rc=$?; echo "config4 rc=$rc"; tail -2 gpurun_out/c4.err; cat gpurun_out/c4.json
[ $rc -ne 0 ] && exit $rc
fi
DA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 --batch 8 --latency-reps 1 --ingest-docs 2 --index-kind ivfflat --ivf-lists 256 --ivf-probes 8 > gpurun_out/tp2.json 2> gpurun_out/tp2.err
rc=$?; echo "tp2 rc=$rc"; tail -4 gpurun_out/tp2.err; cat gpurun_out/tp2.json
[ $rc -ne 0 ] && exit $rc
[ "${RUN_C5:-0}" != 1 ] && exit 0
DA_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 8 --tp 8 --llm llama3-70b --enc bge-large --enc-dtype fp8 --index-kind ivfflat --index-rows 200000 --ivf-lists 256 --ivf-probes 8 --steps 1 --warmup 1 --batch 2 --latency-reps 1 --ingest-docs 0 > gpurun_out/c5.json 2> gpurun_out/c5.err
rc=$?; echo "config5 rc=$rc"; tail -4 gpurun_out/c5.err; cat gpurun_out/c5.json
exit $rc
