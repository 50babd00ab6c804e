#!/bin/bash
# batch-1 decode kernel stats with the VALU (0) and MFMA (1) decode attention
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TAG:-r5m3}
mkdir -p $O
for x in 0 1; do
  (cd /tmp && export TMPDIR=/tmp && DA_DECODE_MFMA1=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/$O/prof_m$x -o p -- python3 $R/bench/decode_prof.py --batch 1 --reps 1 > /dev/null 2> $R/$O/prof_m$x.err) || exit 1
  python bench/kstats_top.py $O/prof_m$x 8 > $O/top_m$x.txt && cat $O/top_m$x.txt
done
