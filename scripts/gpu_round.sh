# Round check: build, all @gpu tests, smoke(), bench.py (1 GPU), rocprofv3 kernel stats of one bench step.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof3
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.err; cat gpurun_out/bench_full.json
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 0 --ingest-docs 0 > $R/gpurun_out/prof3_bench.json 2> $R/gpurun_out/prof3_bench.err
rc=$?
echo "prof rc=$rc"
exit $rc
