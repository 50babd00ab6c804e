set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -k "decode" -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python - <<'PY'
import torch, sys
sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it
for name,B,L,H,Hkv,D in [("phi3_b64",64,2944,32,32,96),("phi3_b32",32,2944,32,32,96),("phi3_b1",1,2944,32,32,96),("llama_b64",64,4096,32,8,128),("l70b_tp8_b64",64,4096,8,1,128)]:
    kc=torch.randn(B,Hkv,4096,D,device='cuda').bfloat16(); vc=torch.randn_like(kc)
    q=torch.randn(B,(H+2*Hkv)*D,device='cuda').bfloat16()
    lens=torch.full((B,),L,device='cuda',dtype=torch.int32); slot=torch.arange(B,device='cuda',dtype=torch.int32)
    for chunk in (0,256,512,1024,2048):
        ms=t(lambda: K.decode_attn(q,kc,vc,lens,slot,H,Hkv,D,max_len=4096,chunk=chunk))
        print(f"{name} chunk={chunk} ms={ms:.3f} TB/s={2*B*Hkv*L*D*2/ms/1e9:.2f}", flush=True)
PY
