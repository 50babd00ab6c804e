set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 400 python - <<'PY' 2>&1 | tee gpurun_out/group.txt
import torch, sys
sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K
def t(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it
for M,N,Kd in [(32768,9216,3072),(32768,16384,3072),(32768,3072,8192),(32768,3072,3072),(8192,8192,8192)]:
    x=(torch.rand(M,Kd,device='cuda')*2-1).bfloat16(); w=((torch.rand(N,Kd,device='cuda')*2-1)*Kd**-0.5).bfloat16()
    fl=2*M*N*Kd; out=[]
    for g in (1,2,4,8,16,32):
        K.lib().da_set_gemm_group(g)
        out.append(f"g{g}={fl/t(lambda: K.gemm(x,w,tile=4,splits=1))/1e9:.0f}")
    K.lib().da_set_gemm_group(4)
    print(f"M={M} N={N} K={Kd} " + " ".join(out), flush=True)
PY
