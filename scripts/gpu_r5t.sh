#!/bin/bash
# Round 5 final tree: 2-rank and 8-rank gloo rehearsals of the N > 1 bench on one GPU, then the deploy stack.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5t
mkdir -p $O
for n in 2 8; do
  T0=$(date +%s)
  DA_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus $n --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
    --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 \
    > $O/bench$n.json 2> $O/bench$n.err || { grep "\[bench\]" $O/bench$n.err | cut -c1-300; tail -5 $O/bench$n.err; exit 1; }
  echo "$n-rank rehearsal wall s: $(( $(date +%s) - T0 ))"
  python -c "
import json,sys; d=json.loads(open('$O/bench$n.json').read().strip().splitlines()[-1])
print({k: (d[k] if not isinstance(d.get(k), dict) else {kk: vv for kk, vv in d[k].items() if kk in ('ok','qps','rows_identical_to_plane','agreement','xgmi_mapped','export_refusals','error')}) for k in ('n_gpus','world_size','ranks_seen','rccl_search','tp_decode','xgmi_allreduce')})
print(d['config']['search_transport'])"
done
STACK_TIMEOUT=500 bash scripts/gpu_stack.sh 64 256 128
