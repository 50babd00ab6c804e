# Round-4 check I: 2-rank self-launched bench (gloo, both ranks on the one GPU), then the kernel GPU
# tests against the -DDA_DEBUG library (device asserts on; built in-tree beforehand with
# python -m docagents_amd.ops.build --debug). usage: bash scripts/gpu_r4i.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4i}; mkdir -p $OUT
DA_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --latency-reps 4 \
  --ingest-batches 1 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench2.json; tail -3 $OUT/bench2.err; [ $rc -ne 0 ] && exit $rc
DA_KERNELS_DEBUG=1 timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_b1_gpu.py \
  tests/test_splitk_fused_gpu.py tests/test_fp16_encoder_gpu.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_debug.log 2>&1
rc=$?; tail -4 $OUT/pytest_debug.log; exit $rc
