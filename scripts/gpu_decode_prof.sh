# Decode-step timing + rocprofv3 kernel stats of the production decoder at batch 1 and batch 64.
# usage: bash scripts/gpu_decode_prof.sh [TAG]   -> gpurun_out/<TAG>/b{1,64}.json, b{1,64}_top.txt
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-decode_prof}; OUT=gpurun_out/$TAG
mkdir -p $OUT
python -m docagents_amd.ops.build > $OUT/build.log 2>&1 || { tail -30 $OUT/build.log; exit 3; }
for B in 1 64; do
  timeout -k 10 300 python bench/decode_prof.py --batch $B > $OUT/b$B.json 2> $OUT/b$B.err || { tail $OUT/b$B.err; exit 4; }
  cat $OUT/b$B.json
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/$OUT/prof_b$B -o p -- python3 $R/bench/decode_prof.py --batch $B --reps 1 > /dev/null 2> $R/$OUT/prof_b$B.err) \
     || { tail $OUT/prof_b$B.err; exit 5; }
  python bench/kstats_top.py $OUT/prof_b$B 25 > $OUT/b${B}_top.txt && cat $OUT/b${B}_top.txt
done
