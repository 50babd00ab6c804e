# Round-4 check H: persistent batch-1 decode vs the per-kernel path after pinning FP contraction
# (probe at 2 / 4 layers, graph vs eager), the decode_b1 GPU tests, then the other new tests and the
# kernel / model / serving suites. usage: bash scripts/gpu_r4h.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4h}; mkdir -p $OUT
for L in 2 4; do
  LAYERS=$L ARMS="b1e:pke,b1g:pkg" STEPS=40 timeout -k 10 300 python -u bench/b1_diverge.py > $OUT/diverge_l$L.txt 2>&1
  rc=$?; grep -E "summary" $OUT/diverge_l$L.txt; [ $rc -ne 0 ] && { tail -20 $OUT/diverge_l$L.txt; exit $rc; }
done
timeout -k 10 600 python -u -m pytest tests/test_decode_b1_gpu.py tests/test_splitk_fused_gpu.py tests/test_index_race_gpu.py \
  tests/test_fp16_encoder_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_new.log 2>&1
rc=$?; tail -8 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_serving_gpu.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_suites.log 2>&1
rc=$?; tail -5 $OUT/pytest_suites.log; exit $rc
