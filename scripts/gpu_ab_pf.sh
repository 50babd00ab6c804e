# Decode GEMM prefetch: numerics, then same-box A/B of the flagship bench (PF=4 default vs PF=1).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_pf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_pf.log
[ $rc -ne 0 ] && exit $rc
for pf in 4 1 4 1; do
  DA_GEMM_PF=$pf timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_pf$pf.json 2>/dev/null || exit 1
  echo "pf=$pf $(python -c "import json;d=json.load(open('gpurun_out/ab_pf$pf.json'));print(d['value'], d['ms_per_step'])")"
done
