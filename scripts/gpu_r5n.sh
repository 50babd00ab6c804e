#!/bin/bash
# Round 5: deploy stack at 128 in flight with the serving engine's batch 64 (default) vs 128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5n
STACK_TIMEOUT=500 bash scripts/gpu_stack.sh 64 512 128 || exit 1
mv gpurun_out/stack_c128.json gpurun_out/r5n/stack_b64.json
ENGINE_MAX_BATCH=128 STACK_TIMEOUT=500 bash scripts/gpu_stack.sh 64 512 128 || exit 1
mv gpurun_out/stack_c128.json gpurun_out/r5n/stack_b128.json
for f in gpurun_out/r5n/stack_b64.json gpurun_out/r5n/stack_b128.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: d.get(k) for k in ('qa_qps','cache_miss_p50_ms','serial_cache_miss_p50_ms','ingest_docs_per_min','query_errors')})" $f
done
