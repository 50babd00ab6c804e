# Round-4 check E: where the persistent batch-1 decode and the per-kernel path part ways (graph
# replay and eager), then the other new GPU tests, the kernel / model / serving suites and the
# 1-GPU bench. usage: bash scripts/gpu_r4e.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4e}; mkdir -p $OUT
GRAPHS=1 timeout -k 10 300 python -u bench/b1_diverge.py > $OUT/diverge_graphs.txt 2>&1
rc=$?; tail -6 $OUT/diverge_graphs.txt; [ $rc -ne 0 ] && exit $rc
GRAPHS=0 timeout -k 10 300 python -u bench/b1_diverge.py > $OUT/diverge_eager.txt 2>&1
rc=$?; tail -6 $OUT/diverge_eager.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_splitk_fused_gpu.py tests/test_index_race_gpu.py tests/test_fp16_encoder_gpu.py \
  -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_new.log 2>&1
rc=$?; tail -12 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_serving_gpu.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_suites.log 2>&1
rc=$?; tail -5 $OUT/pytest_suites.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; cat $OUT/bench1.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench1.err; exit $rc; }
exit 0
