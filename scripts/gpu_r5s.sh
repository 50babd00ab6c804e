#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_allreduce_gpu.py \
  > $O/xgmi.log 2>&1 || { tail -30 $O/xgmi.log; exit 1; }
tail -3 $O/xgmi.log
