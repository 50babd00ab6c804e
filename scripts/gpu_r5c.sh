#!/bin/bash
# round 5: xGMI tests with the visibility probe, the 8-rank rehearsal of bench.py's N > 1 blocks on one
# GPU (gloo ranks sharing the card), then the deploy stack with the serial single-document ingest.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_allreduce_gpu.py \
  > $O/xgmi.log 2>&1 || { tail -30 $O/xgmi.log; exit 1; }
tail -3 $O/xgmi.log
T0=$(date +%s)
DA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
  --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 \
  > $O/bench8.json 2> $O/bench8.err || { tail -30 $O/bench8.err; exit 1; }
echo "8-rank rehearsal wall s: $(( $(date +%s) - T0 ))" | tee $O/bench8.wall
grep "\[bench\]" $O/bench8.err | cut -c1-400
STACK_TIMEOUT=600 bash scripts/gpu_stack.sh 64 256 128
