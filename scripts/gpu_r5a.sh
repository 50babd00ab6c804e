#!/bin/bash
# round 5, first GPU pass: xGMI all-reduce on uncached buffers, the 2-rank rehearsal of the N > 1
# bench blocks (gloo ranks sharing the one GPU), then the 1-GPU headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_allreduce_gpu.py \
  > $O/xgmi.log 2>&1 &&
DA_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --batch 8 --steps 2 --warmup 1 --latency-reps 4 \
  --ingest-docs 8 --ingest-batches 1 --ingest-latency-reps 3 --index-rows 20000 --breakdown 0 \
  > $O/bench2.json 2> $O/bench2.err &&
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > $O/bench1.json 2> $O/bench1.err
