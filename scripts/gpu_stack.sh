# The compose-equivalent multi-process stack on one MI355X (deploy.py: native broker + native KV cache +
# engine server on the GPU + query + gateway + 2 parsers + 2 analyzers, each its own process), driven
# over HTTP by bench/loadgen.py: ingest docs/min, QA throughput, cache-hit latency.
# usage: bash scripts/gpu_stack.sh [docs] [queries] [concurrency]
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 3; }
python -m docagents_amd.native > gpurun_out/native.log 2>&1 || { tail -30 gpurun_out/native.log; exit 3; }
export LLM_PROVIDER=engine MIN_SIMILARITY=-1 LOG_LEVEL=warn TMPDIR=${TMPDIR:-/tmp} INDEX_FSYNC=1
timeout -k 10 1000 python -u bench/loadgen.py --spawn --topology deploy --docs ${1:-64} --words 2000 \
  --queries ${2:-256} --concurrency ${3:-64} > gpurun_out/stack.json 2> gpurun_out/stack.err
rc=$?; echo "stack rc=$rc"; tail -5 gpurun_out/stack.err; cat gpurun_out/stack.json
exit $rc
