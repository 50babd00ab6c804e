#!/bin/bash
# Round 5: QA batch 64 vs 128 on the current kernels (decode at 128 rows runs the 64x128 split-K
# tiles, not gemm_dk), then a kernel-stats profile of the batch-128 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
run() {  # name batch
  echo "== bench B=$2"
  timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 --batch "$2" --latency-reps 4 --ingest-batches 1 \
    --ingest-latency-reps 2 > $O/$1.json 2> $O/$1.err
}
run b64 64 && tail -1 $O/b64.json | cut -c1-300 &&
run b128 128 && tail -1 $O/b128.json | cut -c1-300 &&
echo "== rocprof B=128" &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof128 -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --batch 128 --latency-reps 0 --ingest-batches 1 --ingest-latency-reps 0 \
  --breakdown 0 > $O/prof128.log 2>&1 &&
echo "done"
