# Skinny decode GEMM: numerics (every variant, epilogue, resid+RMSNorm tail), then the cold-weight sweep.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k "gemm or prefetch" --timeout 120 --timeout-method thread > gpurun_out/t_skinny.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_skinny.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench/decode_gemm_sweep.py --shapes phi3,llama8b --m 64,16 > gpurun_out/decode_gemm_sweep.jsonl 2> gpurun_out/decode_gemm_sweep.err
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/decode_gemm_sweep.jsonl; tail -3 gpurun_out/decode_gemm_sweep.err
exit $rc
