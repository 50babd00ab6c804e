# Round-4 check F: persistent batch-1 decode vs the per-kernel path, arm pairs (b1 / pk path x
# e(ager) / g(raph)), every layer's cache rows compared after every step; then the decode_b1 tests.
# usage: bash scripts/gpu_r4f.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4f}; mkdir -p $OUT
ARMS="b1g:b1e,b1e:pke,b1g:pkg" STEPS=24 timeout -k 10 400 python -u bench/b1_diverge.py > $OUT/diverge.txt 2>&1
rc=$?; grep -E "summary|arms" $OUT/diverge.txt; [ $rc -ne 0 ] && { tail -20 $OUT/diverge.txt; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_decode_b1_gpu.py -x -v --timeout 180 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_b1.log 2>&1
rc=$?; tail -8 $OUT/pytest_b1.log; exit $rc
