# Full GPU check: build, every @gpu test, graft smoke().
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
exit $rc
