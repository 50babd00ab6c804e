# MHA decode next-tile prefetch (small batches): numerics, then the chunk sweep with it off / on.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "decode" --timeout 120 --timeout-method thread > gpurun_out/t_dec.log 2>&1 || { tail -30 gpurun_out/t_dec.log; exit 1; }
tail -1 gpurun_out/t_dec.log
for p in 0 128; do
  DA_DECODE_PFT=$p timeout -k 10 300 python bench/decode_chunk_sweep.py > gpurun_out/dec_sweep_pft$p.txt 2>&1 || { tail -20 gpurun_out/dec_sweep_pft$p.txt; exit 1; }
  echo "== DA_DECODE_PFT=$p"; grep "fused=1" gpurun_out/dec_sweep_pft$p.txt | head -3
done
