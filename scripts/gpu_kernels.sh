set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider > gpurun_out/kt.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/kt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench/kernel_bench.py --out gpurun_out/kernel_bench.json > gpurun_out/kb.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -30 gpurun_out/kb.log
exit $rc2
