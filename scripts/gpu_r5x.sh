#!/bin/bash
# Round 5: SEARCH_TRANSPORT=rccl collective plane on device ranks, then the 8-rank gloo rehearsal on one
# GPU with the serving_search block (owner-routed plane vs lock-step collective rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r5x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_collective_plane.py \
  > $O/cplane.log 2>&1 || { tail -30 $O/cplane.log; exit 1; }
tail -2 $O/cplane.log
T0=$(date +%s)
DA_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
  --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 \
  > $O/bench8.json 2> $O/bench8.err || { grep "\[bench\]" $O/bench8.err | cut -c1-300; tail -5 $O/bench8.err; exit 1; }
echo "8-rank rehearsal wall s: $(( $(date +%s) - T0 ))" | tee $O/bench8.wall
grep "serving_search:\|tp_decode:\|rccl_search:\|xgmi_allreduce:" $O/bench8.err | cut -c1-900
