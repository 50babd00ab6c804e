# Kernel-trace the hipBLASLt GEMMs of the sustained bench: kernel names (tile config), VGPRs, LDS, workgroup size.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/blt
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
SECS=0.1 ONLY=ours_w4,ours_w4s5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/blt -o blt -- python3 $R/bench/gemm_sustained.py > $R/gpurun_out/blt.log 2>&1
echo "prof rc=$?"
