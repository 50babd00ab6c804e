set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch 16 --ingest-docs 4 --latency-reps 3 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc2=$?
echo "bench small rc=$rc2"; tail -5 gpurun_out/bench_small.err; cat gpurun_out/bench_small.json
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc3=$?
echo "bench full rc=$rc3"; tail -5 gpurun_out/bench_full.err; cat gpurun_out/bench_full.json
exit $rc3
