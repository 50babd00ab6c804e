#!/bin/bash
# Round 5: batch-1 MHA decode attention on MFMA vs the VALU kernel (A/B), then the decode tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r5m1}
mkdir -p $O
for x in 0 1 0 1; do
  DA_DECODE_MFMA1=$x timeout -k 10 120 python -u bench/decode_mfma1_ab.py >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
B=4 DA_DECODE_MFMA1=0 timeout -k 10 120 python -u bench/decode_mfma1_ab.py >> $O/ab.txt 2>&1 &&
B=4 DA_DECODE_MFMA1=1 timeout -k 10 120 python -u bench/decode_mfma1_ab.py >> $O/ab.txt 2>&1 &&
grep "^{" $O/ab.txt &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "decode" \
  > $O/tests.log 2>&1; tail -3 $O/tests.log
for x in 0 1 0 1; do
  DA_DECODE_MFMA1=$x timeout -k 10 200 python bench/decode_prof.py --batch 1 > $O/b1_m$x.json 2>> $O/b1.err || exit 1
  echo "mfma1=$x $(cat $O/b1_m$x.json)" | tee -a $O/b1.txt
done
