#!/bin/bash
# Round 5: per-shape decode GEMM sweep at 96 / 128 rows (tiles 9 and 2 x splits), weights cold.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 600 python -u bench/decode_gemm_sweep.py --m 128,96 --tiles 9,2 > $O/sweep.txt 2>&1 || { tail -20 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
