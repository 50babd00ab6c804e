# xGMI IPC all-reduce: 2 ranks sharing the box's GPU.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_allreduce_gpu.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/t_ar.log 2>&1
rc=$?
tail -30 gpurun_out/t_ar.log
exit $rc
