# Full agent stack on one MI355X: engine server (GPU) + all-in-one agents (CPU) driven over HTTP.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
python -m docagents_amd.native > gpurun_out/native.log 2>&1 || { cat gpurun_out/native.log; exit 3; }
export MIN_SIMILARITY=-1 LOG_LEVEL=warn
timeout -k 10 900 python -m docagents_amd.services engine --listen tcp://127.0.0.1:19090 > gpurun_out/stack_engine.log 2>&1 &
EPID=$!
ok=0
for i in $(seq 1 240); do
  if python -c "import socket; socket.create_connection(('127.0.0.1', 19090), 1).close()" 2>/dev/null; then ok=1; break; fi
  if ! kill -0 $EPID 2>/dev/null; then break; fi
  sleep 1
done
if [ $ok -ne 1 ]; then echo "engine did not start"; tail -30 gpurun_out/stack_engine.log; kill $EPID 2>/dev/null; exit 1; fi
echo "engine up after ${i}s"
LLM_PROVIDER=engine ENGINE_URL=tcp://127.0.0.1:19090 timeout -k 10 600 python bench/loadgen.py --spawn --docs 128 --words 2000 --queries 256 --concurrency 64 > gpurun_out/loadgen.json 2> gpurun_out/loadgen.err
rc=$?
echo "loadgen rc=$rc"; cat gpurun_out/loadgen.json; tail -5 gpurun_out/loadgen.err
kill $EPID 2>/dev/null
wait $EPID 2>/dev/null
tail -5 gpurun_out/stack_engine.log
exit $rc
