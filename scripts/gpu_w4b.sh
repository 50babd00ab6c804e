set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
SECS=${SECS:-1} ONLY=${ONLY:-ours,ours_w4m1,diag_nodma,hipblaslt} timeout -k 10 400 python bench/gemm_sustained.py 2>&1 | tee gpurun_out/gemm_sus.txt
