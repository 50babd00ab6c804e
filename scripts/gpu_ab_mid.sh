# A/B: 65..1023-row GEMMs on hipBLASLt (DA_BLAS_MID=1, default) vs the in-tree 128x128 tile (=0).
# Flagship (batch 64: only the 261-token shared-head prefill is mid-M) and batch 128 (decode GEMMs M=128).
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/t_mid.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_mid.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_mid.txt
for b in 128 64; do
  for v in 0 1 0 1; do
    DA_BLAS_MID=$v timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --latency-reps 0 --ingest-docs 0 > gpurun_out/ab_mid_one.json 2> gpurun_out/ab_mid_one.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_mid_one.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/ab_mid_one.json'));print('batch=$b DA_BLAS_MID=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ab_mid.txt
  done
done
timeout -k 10 300 python bench.py > gpurun_out/bench_mid.json 2> gpurun_out/bench_mid.err
rc=$?; cat gpurun_out/bench_mid.json; exit $rc
