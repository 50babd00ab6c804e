#!/bin/bash
# Round 5: dense scan with the shared-tile kernel for 17..64 queries (numerics, then 10M x 1024 at
# batch 1 / 16 / 64), then the decode-GEMM sweep at 64..128 rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "topk" \
  > $O/topk.log 2>&1 || { tail -30 $O/topk.log; exit 1; }
tail -2 $O/topk.log
timeout -k 10 300 python -u bench/index_bench.py --kind flat --rows 10000000 --dim 1024 --batches 1,16,64 \
  --out $O/index_flat_10m_1024d.json > $O/index.log 2>&1 || { tail -20 $O/index.log; exit 1; }
cat $O/index.log
timeout -k 10 400 python -u bench/midm_chain.py --ms 64,96,128 \
  --arms blas,auto,2:1,2:2,2:4,8:1,8:2,8:4,9:1,9:2,9:4 > $O/midm.txt 2>&1 || { tail -20 $O/midm.txt; exit 1; }
cat $O/midm.txt
