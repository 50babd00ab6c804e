# BASELINE config 3 (Llama-3-8B summarizer+QA, PDF ingest) and a Llama-3-70B single-GPU run.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 900 python bench.py --llm llama3-8b --pdf-ingest > gpurun_out/bench_llama8b.json 2> gpurun_out/bench_llama8b.err
rc=$?
echo "llama8b rc=$rc"; tail -3 gpurun_out/bench_llama8b.err; cat gpurun_out/bench_llama8b.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1200 python bench.py --llm llama3-70b --enc bge-large --batch 16 --steps 2 --warmup 1 --latency-reps 2 --ingest-docs 4 > gpurun_out/bench_llama70b.json 2> gpurun_out/bench_llama70b.err
rc=$?
echo "llama70b rc=$rc"; tail -3 gpurun_out/bench_llama70b.err; cat gpurun_out/bench_llama70b.json
exit $rc
