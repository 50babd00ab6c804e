#!/bin/bash
# Round 5: same-XCD split exchange of the small-batch decode attention: numerics, microbenchmark, decode step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "decode" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench/decode_xc_ab.py > $O/ab.txt 2>&1 && cat $O/ab.txt | grep "^{" &&
for x in 0 1 0 1; do
  DA_DECODE_XC=$x timeout -k 10 200 python bench/decode_prof.py --batch 1 > $O/b1_xc$x.json 2>> $O/b1.err || exit 1
  echo "xc=$x $(cat $O/b1_xc$x.json)" | tee -a $O/b1.txt
done
