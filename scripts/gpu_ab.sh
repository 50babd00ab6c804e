# Same-box A/B of the flagship bench: lock-step vs ping-pong GEMM schedule.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
for pp in 0 1 0 1; do
  DA_GEMM_PINGPONG=$pp timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_$pp.json 2>/dev/null || exit 1
  echo "pingpong=$pp $(python -c "import json;d=json.load(open('gpurun_out/ab_$pp.json'));print(d['value'], d['ms_per_step'])")"
done
