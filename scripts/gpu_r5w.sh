#!/bin/bash
# same-box A/B: previous library (bench/_ab) vs this one with the tile loop off / on, alternating processes
set -o pipefail
mkdir -p gpurun_out/r5w
for r in 1 2; do
  DA_LIB=bench/_ab/_da_kernels_old.so timeout -k 10 200 python -u bench/gemm_epi_ab.py >> gpurun_out/r5w/ab.txt 2>&1 || exit 1
  DA_GEMM8P_PERSIST=0 timeout -k 10 200 python -u bench/gemm_epi_ab.py >> gpurun_out/r5w/ab.txt 2>&1 || exit 1
  DA_GEMM8P_PERSIST=1 timeout -k 10 200 python -u bench/gemm_epi_ab.py >> gpurun_out/r5w/ab.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm8p or gemm_rope" > gpurun_out/r5w/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5w/bench.txt 2>&1
