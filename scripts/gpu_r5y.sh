#!/bin/bash
# Round 5: the 8-rank gloo rehearsal with and without the serving_search block (does the block slow
# the later tp_decode / xgmi blocks when 8 ranks share one GPU?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5y
mkdir -p $O
for n in 256 0; do
  T0=$(date +%s)
  DA_DIST_BACKEND=gloo timeout -k 10 450 python bench.py --gpus 8 --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
    --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 --serving-requests $n \
    > $O/bench8_s$n.json 2> $O/bench8_s$n.err || { grep "\[bench\]" $O/bench8_s$n.err | cut -c1-300; tail -5 $O/bench8_s$n.err; exit 1; }
  echo "serving_requests=$n wall s: $(( $(date +%s) - T0 ))" | tee -a $O/walls.txt
  grep -o "serving_search: .\{0,300\}\|b1_decode_ms_per_step': [0-9.]*\|'16KB': {'xgmi': [0-9.]*" $O/bench8_s$n.err
done
