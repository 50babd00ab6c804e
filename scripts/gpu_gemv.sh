set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or gemv" -p no:cacheprovider > gpurun_out/t_gemv.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t_gemv.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python - <<'PY' 2>&1 | tee gpurun_out/gemv_bench.txt
import torch, sys
sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K
def t(fn, it=100):
    for _ in range(5): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it
for name,N,Kd,epi in [("phi3_qkv",9216,3072,0),("phi3_o",3072,3072,4),("phi3_gu",16384,3072,3),("phi3_down",3072,8192,4),("phi3_lm",32064,3072,0),
                      ("llama8b_gu",28672,4096,3),("llama8b_down",4096,14336,4),("llama70b_gu",57344,8192,3),("llama70b_down",8192,28672,4),("llama70b_qkv",10240,8192,0)]:
    x=torch.randn(1,Kd,device='cuda').bfloat16(); w=(torch.randn(N,Kd,device='cuda')*Kd**-0.5).bfloat16()
    r=torch.randn(1,N,device='cuda').bfloat16() if epi==4 else None
    by=N*Kd*2
    t_old=t(lambda: K.gemm(x,w,epi=epi,resid=r,tile=3,splits=K._auto_splits(1,N,Kd)))
    t_new=t(lambda: K.gemm(x,w,epi=epi,resid=r,tile=6,splits=1))
    print(f"{name} N={N} K={Kd}: splitk {t_old*1e3:.1f}us ({by/t_old/1e9:.2f} TB/s)  gemv {t_new*1e3:.1f}us ({by/t_new/1e9:.2f} TB/s)", flush=True)
PY
