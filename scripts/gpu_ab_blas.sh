# Same-box A/B of the flagship bench: prefill plain GEMMs on gemm256 (0) vs hipBLASLt (1).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "gemm" > gpurun_out/t_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_gemm.log
[ $rc -ne 0 ] && exit $rc
for b in 0 1 0 1; do
  DA_BLAS_PREFILL=$b timeout -k 10 600 python bench.py --latency-reps 0 --ingest-docs 0 > gpurun_out/abb_$b.json 2>/dev/null || exit 1
  echo "blas=$b $(python -c "import json;d=json.load(open('gpurun_out/abb_$b.json'));print(d['value'], d['ms_per_step'])")"
done
