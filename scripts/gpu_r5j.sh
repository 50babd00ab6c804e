#!/bin/bash
# Round 5: dense scan (radix-select cuts, per-lane sub-buffers) numerics + probe + index bench;
# 65..128-row decode GEMMs on the 128x64 tile (numerics, chain sweep), then bench at batch 128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "topk or gemm_decode_tile or resid_rmsnorm or mid_m or gemm_rope or flash_attn or kv_from_cache" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
timeout -k 10 300 python -u bench/scan_probe.py --qs 1,16,17,64 > $O/scan_probe.txt 2>&1 || { tail -20 $O/scan_probe.txt; exit 1; }
cat $O/scan_probe.txt
timeout -k 10 300 python -u bench/index_bench.py --kind flat --rows 10000000 --dim 1024 --batches 1,16,64 \
  --out $O/index_flat_10m_1024d.json > $O/index.log 2>&1 || { tail -20 $O/index.log; exit 1; }
cat $O/index.log
timeout -k 10 300 python -u bench/midm_chain.py --ms 96,128 --arms blas,auto,9:2,9:4,9:8 > $O/midm.txt 2>&1 || { tail -20 $O/midm.txt; exit 1; }
cat $O/midm.txt
timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 --batch 128 --latency-reps 4 --ingest-batches 1 \
  --ingest-latency-reps 2 > $O/b128.json 2> $O/b128.err || { tail -20 $O/b128.err; exit 1; }
tail -1 $O/b128.json | cut -c1-300
