# Round-4 check G: persistent vs per-kernel batch-1 decode at 1 / 2 / 4 layers (attention output,
# residual, cache rows compared every step). usage: bash scripts/gpu_r4g.sh TAG
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4g}; mkdir -p $OUT
for L in 1 2 4; do
  LAYERS=$L ARMS="b1e:pke" STEPS=40 timeout -k 10 300 python -u bench/b1_diverge.py > $OUT/diverge_l$L.txt 2>&1
  rc=$?; grep -E "summary" $OUT/diverge_l$L.txt; [ $rc -ne 0 ] && { tail -20 $OUT/diverge_l$L.txt; exit $rc; }
done
exit 0
