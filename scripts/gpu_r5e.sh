#!/bin/bash
# round 5: the dense scan with per-query candidate buffers (numerics + 10M x 1024 timing at batch 1 /
# 16 / 64), the 8-rank rehearsal (TP verdict decoder chosen per world), then the deploy stack (port
# block below the ephemeral range).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "topk" \
  > $O/topk.log 2>&1 || { tail -30 $O/topk.log; exit 1; }
tail -2 $O/topk.log
timeout -k 10 300 python -u bench/index_bench.py --kind flat --rows 10000000 --dim 1024 --batches 1,16,64 \
  --out $O/index_flat_10m_1024d.json > $O/index.log 2>&1 || { tail -20 $O/index.log; exit 1; }
cat $O/index.log
T0=$(date +%s)
DA_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
  --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 \
  > $O/bench8.json 2> $O/bench8.err || { grep "\[bench\]" $O/bench8.err | cut -c1-300; exit 1; }
echo "8-rank rehearsal wall s: $(( $(date +%s) - T0 ))" | tee $O/bench8.wall
grep "tp_decode" $O/bench8.err | cut -c1-400
STACK_TIMEOUT=600 bash scripts/gpu_stack.sh 64 256 128
