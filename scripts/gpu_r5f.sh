#!/bin/bash
# Round 5: dense scan with L2-resident rows for several query blocks (10M x 1024 at batch 1/16/64),
# QA batch 64 vs 128 on the current kernels, a 4-rank rehearsal (TP verdict on tiny-dec-tp8), then a
# kernel-stats profile of the batch-128 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 300 python -u bench/index_bench.py --kind flat --rows 10000000 --dim 1024 --batches 1,16,64 \
  --out $O/index_flat_10m_1024d.json > $O/index.log 2>&1 || { tail -20 $O/index.log; exit 1; }
cat $O/index.log
run() {  # name batch
  echo "== bench B=$2"
  timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 --batch "$2" --latency-reps 4 --ingest-batches 1 \
    --ingest-latency-reps 2 > $O/$1.json 2> $O/$1.err
}
run b64 64 && tail -1 $O/b64.json | cut -c1-300 &&
run b128 128 && tail -1 $O/b128.json | cut -c1-300 || exit 1
T0=$(date +%s)
DA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --batch 4 --steps 1 --warmup 1 --latency-reps 2 \
  --ingest-docs 4 --ingest-batches 1 --ingest-latency-reps 2 --index-rows 20000 --breakdown 0 \
  > $O/bench4.json 2> $O/bench4.err || { grep "\[bench\]" $O/bench4.err | cut -c1-300; exit 1; }
echo "4-rank rehearsal wall s: $(( $(date +%s) - T0 ))"
grep "tp_decode" $O/bench4.err | cut -c1-600
echo "== rocprof B=128" &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof128 -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --batch 128 --latency-reps 0 --ingest-batches 1 --ingest-latency-reps 0 \
  --breakdown 0 > $O/prof128.log 2>&1 &&
echo "done"
