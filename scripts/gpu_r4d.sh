# Round-4 check D: the 1-GPU bench, the persistent batch-1 decode A/B vs the per-kernel path, and a
# rocprofv3 kernel-stats profile of one bench step. usage: bash scripts/gpu_r4d.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4d}; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; cat $OUT/bench1.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench1.err; exit $rc; }
timeout -k 10 300 python -u bench/b1_persistent_ab.py > $OUT/b1_persistent_ab.txt 2>&1
rc=$?; tail -4 $OUT/b1_persistent_ab.txt; [ $rc -ne 0 ] && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 2 --ingest-docs 16 --breakdown 0 > $R/$OUT/prof_bench.json 2> $R/$OUT/prof_bench.err)
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/prof_bench.err; exit $rc; }
python bench/kstats_top.py $OUT/prof 25 > $OUT/kstats_top.txt 2>&1; head -26 $OUT/kstats_top.txt
gzip -f $OUT/prof/*kernel_trace.csv
exit 0
