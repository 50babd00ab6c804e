#!/bin/bash
# Round 5: QKV epilogue k / v to the cache only + attention from the cache (kv_out 0) vs round 4's
# second copy in the qkv tile (kv_out 1): timing, then PMC passes per arm.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 300 python -u bench/qkv_rope_ab.py --reps 20 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for arm in 0 1; do
  bash scripts/gpu_pmc.sh r5l/pmc_kv$arm bench/qkv_rope_ab.py --arm $arm --reps 3 || exit 1
done
FILTER=gemm8p python bench/pmc_summary.py r5l/pmc_kv0 r5l/pmc_kv1
FILTER=flash_attn python bench/pmc_summary.py r5l/pmc_kv0 r5l/pmc_kv1
