set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "rope or decode" -p no:cacheprovider > gpurun_out/t_dec.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t_dec.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench/decode_bench.py --out gpurun_out/decode_bench.json > gpurun_out/decode_bench.log 2>&1
rc=$?
echo "bench rc=$rc"; cat gpurun_out/decode_bench.log
exit $rc
