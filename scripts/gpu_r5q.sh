#!/bin/bash
# Round 5: per-shape decode tile/split choice at 65..128 rows: numerics, chain, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py \
  -k "gemm or decode or generate" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
timeout -k 10 300 python -u bench/midm_chain.py --ms 96,128 --arms blas,auto,9:4 > $O/midm.txt 2>&1 || { tail -20 $O/midm.txt; exit 1; }
cat $O/midm.txt
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','p50_cache_miss_ms','ingest_docs_per_min','ingest_docs_per_min_runs','qa_step_phase_ms','ingest_phase_ms')})"
