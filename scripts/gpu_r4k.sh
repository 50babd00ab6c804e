# Round-4 check K: the batch-1 merged O projection (attention partials merged on the O GEMV's
# input load): its GPU tests + the decode-attention / persistent-decode regressions, then the
# batch-1 decode-step A/B over the merged GEMV's workgroup shapes. usage: bash scripts/gpu_r4k.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4k}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_o_merge_gpu.py tests/test_decode_b1_gpu.py > $OUT/pytest_omerge.log 2>&1
rc=$?; tail -3 $OUT/pytest_omerge.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest_omerge.log | head -20; exit $rc; }
SHAPES=${SHAPES:-81,82,161} timeout -k 10 400 python -u bench/o_merge_ab.py > $OUT/o_merge_ab.txt 2>&1
rc=$?; tail -2 $OUT/o_merge_ab.txt; exit $rc
