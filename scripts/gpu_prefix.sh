# Shared-prompt-head prefill: kernel + model tests, then flagship A/B (DA_SHARE_PREFIX=0/1).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_pre.log 2>&1 || { tail -30 gpurun_out/t_pre.log; exit 1; }
tail -1 gpurun_out/t_pre.log
for v in 0 1 0 1; do
  DA_SHARE_PREFIX=$v timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_pre$v.json 2>/dev/null || exit 1
  echo "share_prefix=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_pre$v.json'));print(d['value'], d['ms_per_step'], d['prefill_tokens'])")"
done
