# Causal flash attention longest-first dispatch: numerics, then same-box A/B of the flagship bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "flash" --timeout 120 --timeout-method thread > gpurun_out/t_fl.log 2>&1 || { tail -30 gpurun_out/t_fl.log; exit 1; }
tail -1 gpurun_out/t_fl.log
for v in 1 0 1 0; do
  DA_FLASH_REV=$v timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_rev$v.json 2>/dev/null || exit 1
  echo "flash_rev=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_rev$v.json'));print(d['value'], d['ms_per_step'])")"
done
