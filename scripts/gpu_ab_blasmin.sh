# p50 latency A/B: prefill GEMMs of a batch-1 prompt (M ~ 2.9k) on hipBLASLt (DA_BLAS_MIN_M=1024) vs the hand-written tiles.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 4096 1024 4096 1024; do
  DA_BLAS_MIN_M=$v timeout -k 10 600 python bench.py --steps 1 --warmup 1 --latency-reps 9 --ingest-docs 0 > gpurun_out/ab_bm$v.json 2>/dev/null || exit 1
  echo "blas_min_m=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_bm$v.json'));print(d['value'], d['p50_cache_miss_ms'])")"
done
