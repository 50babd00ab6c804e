# 256x256 GEMMs: numerics, then sustained throughput vs hipBLASLt.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "gemm" > gpurun_out/t_w4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_w4.log
[ $rc -ne 0 ] && exit $rc
SECS=${SECS:-1} ONLY=${ONLY:-ours,ours_w4m1,ours_w4m3,diag_nodma,hipblaslt} timeout -k 10 400 python bench/gemm_sustained.py 2>&1 | tee gpurun_out/gemm_sus.txt
