set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 0 --ingest-docs 0 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err
rc=$?
echo "rc=$rc"; tail -3 $R/gpurun_out/prof_bench.err
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
