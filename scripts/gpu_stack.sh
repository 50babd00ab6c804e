# The compose-equivalent multi-process stack on one MI355X (deploy.py: native broker + native KV cache +
# engine server on the GPU + query + gateway + 2 parsers + 2 analyzers, each its own process), driven
# over HTTP by bench/loadgen.py: ingest docs/min, QA throughput, cache-hit latency, plus a "diag"
# block (per-service handler means, engine GPU-thread time per command, batching counters).
# usage: bash scripts/gpu_stack.sh [docs] [queries] ["concurrency ..."]   -> gpurun_out/stack_c<C>.json
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 3; }
python -m docagents_amd.native > gpurun_out/native.log 2>&1 || { tail -30 gpurun_out/native.log; exit 3; }
mkdir -p gpurun_out/stack_tmp
# the stack's sqlite / index / supervisor logs land under gpurun_out so a failing service's log comes back
export LLM_PROVIDER=engine MIN_SIMILARITY=-1 LOG_LEVEL=warn TMPDIR=$R/gpurun_out/stack_tmp INDEX_FSYNC=1
for C in ${3:-64}; do
  timeout -k 10 ${STACK_TIMEOUT:-600} python -u bench/loadgen.py --spawn --topology deploy --docs ${1:-64} \
    --words 2000 --queries ${2:-256} --concurrency $C > gpurun_out/stack_c$C.json 2> gpurun_out/stack_c$C.err
  rc=$?; echo "stack c=$C rc=$rc"; tail -5 gpurun_out/stack_c$C.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); d.pop('diag',None); print(json.dumps(d))" gpurun_out/stack_c$C.json
  [ $rc -eq 0 ] || exit $rc
done
