#!/bin/bash
# persistent GEMM with the previous tile's stores in flight under K-tile 0: numerics, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm8p or gemm_rope or test_gemm" tests/test_fp16_encoder_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/gemm_persist_ab.py > $O/ab.txt 2>&1 && grep summary $O/ab.txt | cut -c1-2500 &&
timeout -k 10 500 python -u bench/gemm_ab.py 7,blas > $O/gemm_ab.txt 2>&1 && grep -v check $O/gemm_ab.txt | grep "^{" | cut -c1-80
