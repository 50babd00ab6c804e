#!/bin/bash
# graphed one-sequence encoder: numerics, then the engine-level latency phases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5eg
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py -k "encoder" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_serving_gpu.py > $O/serving.log 2>&1 || { tail -30 $O/serving.log; exit 1; }
tail -2 $O/serving.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && python -c "
import json; b=json.load(open('$O/bench.json')); print(b['value'], b['p50_cache_miss_ms'], b['latency_phase_ms'])"
