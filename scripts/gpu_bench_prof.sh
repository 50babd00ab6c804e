set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof2
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.err; cat gpurun_out/bench_full.json
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2 -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 0 --ingest-docs 0 > $R/gpurun_out/prof2_bench.json 2> $R/gpurun_out/prof2_bench.err
rc=$?
echo "prof rc=$rc"
exit $rc
