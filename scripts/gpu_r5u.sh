#!/bin/bash
# persistent gemm8p: numerics (persistent vs fp32 reference and vs one workgroup per tile) + A/B timing
set -o pipefail
mkdir -p gpurun_out/r5u
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm8p or gemm_rope or test_gemm" tests/test_fp16_encoder_gpu.py > gpurun_out/r5u/tests.log 2>&1 &&
timeout -k 10 300 python -u bench/gemm_persist_ab.py > gpurun_out/r5u/ab.txt 2>&1
