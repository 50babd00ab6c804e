set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k gemm -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python - <<'PY'
import torch, sys
sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K
def t(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it
for M,N,Kd in [(4096,9216,3072),(32768,9216,3072),(32768,16384,3072),(32768,3072,8192),(8192,8192,8192),(65536,768,3072)]:
    x=(torch.rand(M,Kd,device='cuda')*2-1).bfloat16(); w=((torch.rand(N,Kd,device='cuda')*2-1)*Kd**-0.5).bfloat16()
    fl=2*M*N*Kd
    out=[]
    ref=None
    for sch in range(2):
        K.lib().da_set_gemm_pingpong(sch)
        tf=fl/t(lambda: K.gemm(x,w,tile=4,splits=1))/1e9
        o=K.gemm(x,w,tile=4,splits=1).float()
        ref = o if ref is None else ref
        out.append(f"s{sch}={tf:.0f}({(o-ref).abs().max().item():.1g})")
        tf=fl/t(lambda: K.gemm(x,w,epi=K.EPI_SWIGLU,tile=4,splits=1))/1e9
        out.append(f"sw{sch}={tf:.0f}")
    K.lib().da_set_gemm_pingpong(0)
    tt=fl/t(lambda: torch.matmul(x,w.t()))/1e9
    print(f"M={M} N={N} K={Kd} " + " ".join(out) + f" hipblaslt={tt:.0f}", flush=True)
PY
