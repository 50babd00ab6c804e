# Round-4 check F: persistent batch-1 decode vs the per-kernel path, arm pairs (b1 / pk path x
# e(ager) / g(raph)) to separate a path's own nondeterminism from a mismatch between paths, then the
# index race tests. usage: bash scripts/gpu_r4f.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4f}; mkdir -p $OUT
ARMS="pke:pke,b1e:b1e,b1e:pke,b1g:b1e,pkg:pke" STEPS=24 timeout -k 10 400 python -u bench/b1_diverge.py > $OUT/diverge.txt 2>&1
rc=$?; grep -E "summary|arms" $OUT/diverge.txt; [ $rc -ne 0 ] && { tail -20 $OUT/diverge.txt; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_index_race_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_race.log 2>&1
rc=$?; tail -8 $OUT/pytest_race.log; exit $rc
