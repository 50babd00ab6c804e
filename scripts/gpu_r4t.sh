# Round-4 final profile: rocprofv3 kernel-trace stats of one bench step on the final tree (the
# summary lands in profiles/r4/final_prof/ after the run). usage: bash scripts/gpu_r4t.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4t}; mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 2 --ingest-docs 16 --breakdown 0 > $R/$OUT/prof_bench.json 2> $R/$OUT/prof_bench.err)
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/prof_bench.err; exit $rc; }
python bench/kstats_top.py $OUT/prof 30 > $OUT/kstats_top.txt 2>&1; head -31 $OUT/kstats_top.txt
rm -f $OUT/prof/*kernel_trace.csv
exit 0
