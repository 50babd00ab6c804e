# p50 A/B: plain GEMMs of 1024..4095 rows that underfill the 256x256 tile on hipBLASLt (1) vs the hand tiles (0).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_uf.log 2>&1 || { tail -30 gpurun_out/t_uf.log; exit 1; }
tail -1 gpurun_out/t_uf.log
for v in 1 0 1 0; do
  DA_BLAS_UNDERFILL=$v timeout -k 10 600 python bench.py --steps 2 --warmup 1 --latency-reps 9 --ingest-docs 32 > gpurun_out/ab_uf$v.json 2>/dev/null || exit 1
  echo "underfill_blas=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_uf$v.json'));print(d['value'], d['p50_cache_miss_ms'], d['ingest_docs_per_min'])")"
done
