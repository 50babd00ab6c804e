# Round-4 check C: new GPU tests (persistent batch-1 decode, fused split-K, index race), the model /
# kernel GPU suites they touch, then the 1-GPU bench and a 2-rank self-launched bench (gloo).
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4c}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_decode_b1_gpu.py tests/test_splitk_fused_gpu.py tests/test_index_race_gpu.py tests/test_fp16_encoder_gpu.py \
  -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_new.log 2>&1
rc=$?; tail -12 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_serving_gpu.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_suites.log 2>&1
rc=$?; tail -5 $OUT/pytest_suites.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; cat $OUT/bench1.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench1.err; exit $rc; }
DA_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --latency-reps 4 \
  --ingest-batches 1 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench2.json; tail -5 $OUT/bench2.err; exit $rc
