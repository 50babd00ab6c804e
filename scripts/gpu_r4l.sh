# Round-4 check L: per-kernel times of the batch-1 decode step with the ticketed attention merge
# vs the merged O projection (two rocprofv3 --kernel-trace --stats runs of bench/o_merge_ab.py,
# one arm each). usage: bash scripts/gpu_r4l.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4l}; mkdir -p $OUT
for arm in ticket merge; do
  if [ $arm = ticket ]; then T=1; S=0; else T=0; S=${MSHAPE:-82}; fi
  (cd /tmp && export TMPDIR=/tmp && TICKET=$T SHAPES=$S ROUNDS=1 STEPS=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$arm -o run -- python3 $R/bench/o_merge_ab.py > $R/$OUT/ab_$arm.txt 2>&1)
  rc=$?; echo "$arm rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/ab_$arm.txt; exit $rc; }
  python bench/kstats_top.py $OUT/prof_$arm 14 > $OUT/kstats_$arm.txt 2>&1; cat $OUT/kstats_$arm.txt
  rm -f $OUT/prof_$arm/*kernel_trace.csv
done
exit 0
