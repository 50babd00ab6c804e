set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench/kernel_bench.py --out gpurun_out/kernel_bench.json > gpurun_out/kb.log 2>&1
rc=$?
echo "kbench rc=$rc"; grep -E "decode|prefill'|swiglu" gpurun_out/kb.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.err; cat gpurun_out/bench_full.json
exit $rc
