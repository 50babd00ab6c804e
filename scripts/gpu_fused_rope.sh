# Fused RoPE decode: numerics (kernels + models), decode sweep, same-box A/B of the flagship bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_fr.log 2>&1 || { tail -30 gpurun_out/t_fr.log; exit 1; }
tail -1 gpurun_out/t_fr.log
for v in 1 0 1 0; do
  DA_FUSED_ROPE=$v timeout -k 10 600 python bench.py --latency-reps 5 --ingest-docs 0 > gpurun_out/ab_fr$v.json 2>/dev/null || exit 1
  echo "fused_rope=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_fr$v.json'));print(d['value'], d['ms_per_step'], d['p50_cache_miss_ms'])")"
done
