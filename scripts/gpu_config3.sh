# BASELINE config 3: Llama-3-8B summarizer + QA with PDF ingest (gateway PDF extraction in the timed ingest path).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --llm llama3-8b --pdf-ingest > gpurun_out/c3.json 2> gpurun_out/c3.err
rc=$?; echo "config3 rc=$rc"; tail -2 gpurun_out/c3.err; cat gpurun_out/c3.json
exit $rc
