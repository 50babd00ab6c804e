# Same-box A/B of the flagship bench: gate/up GEMM on gemm256 (fused SwiGLU) vs hipBLASLt + SwiGLU pass.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "swiglu" --timeout 120 --timeout-method thread > gpurun_out/t_sw.log 2>&1 || { tail -20 gpurun_out/t_sw.log; exit 1; }
tail -1 gpurun_out/t_sw.log
for v in 0 1 0 1; do
  DA_BLAS_SWIGLU=$v timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_sw$v.json 2>/dev/null || exit 1
  echo "blas_swiglu=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_sw$v.json'));print(d['value'], d['ms_per_step'])")"
done
