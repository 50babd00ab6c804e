# Round-4 check B: persistent batch-1 decode tests, index race tests, 1-GPU bench, then a 2-rank
# self-launched bench (gloo, both ranks on the one GPU). usage: bash scripts/gpu_r4b.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4b}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_b1_gpu.py tests/test_index_race_gpu.py -x -v --timeout 180 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; cat $OUT/bench1.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench1.err; exit $rc; }
DA_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --latency-reps 4 \
  --ingest-batches 1 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench2.json; tail -5 $OUT/bench2.err; exit $rc
