# Stream-overlap probe: decode attention (HBM-bound) vs prefill GEMM (MFMA-bound) on two streams.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/overlap.jsonl
for g in own torch; do
  timeout -k 10 120 python bench/overlap_probe.py --gemm $g --out gpurun_out/overlap.jsonl || exit $?
done
timeout -k 10 120 python bench/overlap_probe.py --gemm own --batch 64 --m 8192 --out gpurun_out/overlap.jsonl || exit $?
