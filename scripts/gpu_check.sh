# Round check on one MI355X: build, @gpu tests, smoke(), flagship bench, rocprofv3 kernel stats of
# one bench step (+ optional extra command). usage: bash scripts/gpu_check.sh TAG ["extra cmd"]
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-check}; EXTRA=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
python -m docagents_amd.ops.build > $OUT/build.log 2>&1 || { tail -30 $OUT/build.log; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 1 --ingest-docs 16 --breakdown 0 > $R/$OUT/prof_bench.json 2> $R/$OUT/prof_bench.err)
rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
python - <<PY
import csv, glob
f = glob.glob("$OUT/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("Cijk kernels:", sum(1 for r in rows if "Cijk" in r["Name"]))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["Percentage"]):6.2f}%  {int(r["Calls"]):6d}  {r["Name"][:90]}')
PY
# the per-dispatch trace is tens of MB: compressed, so the merged gpurun_out stays under its cap
gzip -f $OUT/prof/*kernel_trace.csv
if [ -n "$EXTRA" ]; then eval "$EXTRA"; fi
