# Round-4 check O: the 33..64-row QKV reduce folded into the decode attention — its GPU tests, the
# batch-64 decode-step A/B, and per-kernel stats of one arm each. usage: bash scripts/gpu_r4o.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4o}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_qkv_fold_gpu.py > $OUT/pytest_qkv_fold.log 2>&1
rc=$?; tail -3 $OUT/pytest_qkv_fold.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest_qkv_fold.log | head -20; exit $rc; }
timeout -k 10 500 python -u bench/qkv_fold_ab.py > $OUT/qkv_fold_ab.txt 2>&1
rc=$?; tail -2 $OUT/qkv_fold_ab.txt; exit $rc
