#!/bin/bash
# Round 5: decode GEMMs at 65..128 rows (32-layer Phi-3 projection chain, graph-replayed): the
# production route vs the 64x128 tile at fixed splits vs the 128x128 / 128x64 PF4 tiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 400 python -u bench/midm_chain.py --ms 64,96,128 \
  --arms blas,auto,2:1,2:2,2:4,8:1,8:2,8:4,9:1,9:2,9:4 > $O/midm.txt 2>&1 || { tail -20 $O/midm.txt; exit 1; }
cat $O/midm.txt
