# GEMM A/B + PMC: bash scripts/gpu_gemm_ab.sh "ARMS" "PMC_ARMS"
#   ARMS: comma list for bench/gemm_ab.py (e.g. 7:0,7:2,blas; "" skips the A/B)
#   PMC_ARMS: space list of ARM values for bench/gemm_one.py counter passes (e.g. "7:2 blas")
set -u
R=$GRAFT_REPO_ROOT
cd $R
ARMS=${1:-}
PMC=${2:-}
if [ -n "$ARMS" ]; then
  timeout -k 10 400 python bench/gemm_ab.py $ARMS > gpurun_out/gemm_ab.txt 2>&1 || { tail -20 gpurun_out/gemm_ab.txt; exit 1; }
  grep shape gpurun_out/gemm_ab.txt | cut -c1-160
fi
for a in $PMC; do
  ARM=$a bash scripts/gpu_pmc.sh pmc_${a//:/_} bench/gemm_one.py || exit 1
done
