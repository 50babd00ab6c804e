set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "topk or kmeans" -p no:cacheprovider > gpurun_out/t_ix.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t_ix.log
if [ $rc -ne 0 ]; then if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench/index_bench.py --kind ivfflat --rows 100000000 --dim 1024 --lists 8192 --probes 8,32,128 --batches 1,64 --out gpurun_out/index_ivf100m.json > gpurun_out/index_ivf100m.log 2>&1
rc=$?; echo "ivf100m rc=$rc"; cat gpurun_out/index_ivf100m.log | tail -6
exit $rc; fi
timeout -k 10 600 python bench/index_bench.py --kind ivfflat --rows 10000000 --dim 1024 --lists 4096 --probes 4,16,64 --out gpurun_out/index_ivf10m.json > gpurun_out/index_ivf10m.log 2>&1
rc=$?; echo "ivf rc=$rc"; cat gpurun_out/index_ivf10m.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench/index_bench.py --kind ivfflat --rows 100000000 --dim 1024 --lists 8192 --probes 8,32,128 --batches 1,64 --out gpurun_out/index_ivf100m.json > gpurun_out/index_ivf100m.log 2>&1
rc=$?; echo "ivf100m rc=$rc"; cat gpurun_out/index_ivf100m.log | tail -6
exit $rc
