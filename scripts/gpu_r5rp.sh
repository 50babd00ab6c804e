#!/bin/bash
# persistent RoPE-epilogue GEMM: numerics then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5rp
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_rope or gemm8p_persistent" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/gemm_persist_ab.py > $O/ab.txt 2>&1 && grep rope $O/ab.txt | head -2
