# Sustained GEMM throughput (ours vs ping-pong vs hipBLASLt) + hipBLASLt kernel names via kernel trace.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/blt
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python bench/gemm_sustained.py 2>&1 | tee gpurun_out/gemm_sus.txt
rc=$?
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
SECS=0.2 ONLY=hipblaslt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/blt -o blt -- python3 $R/bench/gemm_sustained.py > $R/gpurun_out/blt.log 2>&1
echo "prof rc=$?"
