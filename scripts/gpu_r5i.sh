#!/bin/bash
# Round 5: dense scan with radix-select top-K cuts: numerics, then the probe (streaming vs top-K
# bookkeeping) and the index bench on 10M x 1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "topk" \
  > $O/topk.log 2>&1 || { tail -30 $O/topk.log; exit 1; }
tail -2 $O/topk.log
timeout -k 10 300 python -u bench/scan_probe.py > $O/scan_probe.txt 2>&1 || { tail -20 $O/scan_probe.txt; exit 1; }
cat $O/scan_probe.txt
timeout -k 10 300 python -u bench/index_bench.py --kind flat --rows 10000000 --dim 1024 --batches 1,16,64 \
  --out $O/index_flat_10m_1024d.json > $O/index.log 2>&1 || { tail -20 $O/index.log; exit 1; }
cat $O/index.log
