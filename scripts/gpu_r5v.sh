#!/bin/bash
# Round 5: gemm8p with W as the MFMA A operand (8-B staging writes): numerics, then A/B vs the
# previous library at the prefill epilogues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_encoder_gpu.py tests/test_models_gpu.py \
  -k "gemm or rope or kv_from_cache or fp16 or encoder or prefill or generate" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
export DA_BUILD_ON_IMPORT=0
for i in 1 2; do
  DA_LIB=$PWD/bench/_ab/_da_kernels_old.so timeout -k 10 200 python -u bench/gemm_epi_ab.py >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
  timeout -k 10 200 python -u bench/gemm_epi_ab.py >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep "^{" $O/ab.txt
