# Round-4 check X: flash prefill kernel time in situ (Llama-3-8B QA bench step) with the XCD-grouped
# dispatch (rev 3) vs grid order (rev 1): rocprofv3 kernel stats of one reduced bench run each.
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4x}; mkdir -p $OUT
for rev in 3 1; do
  (cd /tmp && export TMPDIR=/tmp && DA_FLASH_REV=$rev timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$rev -o b -- python3 $R/bench.py --llm ${LLM:-llama3-8b} --steps 1 --warmup 1 --latency-reps 1 --ingest-docs 0 --breakdown 0 > $R/$OUT/b_$rev.json 2> $R/$OUT/b_$rev.err)
  rc=$?; echo "rev $rev rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/b_$rev.err; exit $rc; }
  python bench/kstats_top.py $OUT/prof_$rev 12 > $OUT/kstats_$rev.txt 2>&1; grep -E "flash|total" $OUT/kstats_$rev.txt
  rm -f $OUT/prof_$rev/*kernel_trace.csv
done
exit 0
