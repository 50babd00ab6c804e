set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/proflat
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/proflat -o lat -- python3 $R/bench.py --batch 1 --steps 4 --warmup 1 --latency-reps 0 --ingest-docs 0 > $R/gpurun_out/proflat.json 2> $R/gpurun_out/proflat.err
rc=$?
echo "prof rc=$rc"; cat $R/gpurun_out/proflat.json
exit $rc
