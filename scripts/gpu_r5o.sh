#!/bin/bash
# Round 5: the default bench (batch 128, ingest batches of 128 docs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','p50_cache_miss_ms','ingest_docs_per_min','ingest_docs_per_min_runs','ingest_single_doc_p50_ms','ingest_phase_ms')})"
