# Round-4 check J: batch-1 decode attention with 8 waves per workgroup (numerics test + microbench).
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4j}; mkdir -p $OUT
CHUNKS=768 timeout -k 10 300 python -u bench/decode_w8.py > $OUT/decode_w8.txt 2>&1
rc=$?; cat $OUT/decode_w8.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "decode" -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest_w8.log 2>&1
rc=$?; tail -3 $OUT/pytest_w8.log; exit $rc
