set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "fp8 or gemm" -p no:cacheprovider > gpurun_out/t_fp8.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t_fp8.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python - <<'PY'
import torch, sys
sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K
def t(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it
for M,N,Kd in [(65536,2304,768),(65536,768,768),(65536,3072,768),(65536,768,3072),(32768,9216,3072),(8192,8192,8192)]:
    x=(torch.rand(M,Kd,device='cuda')*2-1).bfloat16(); w=((torch.rand(N,Kd,device='cuda')*2-1)*Kd**-0.5).bfloat16()
    fl=2*M*N*Kd
    tb=t(lambda: K.gemm(x,w))
    xq,sa=K.quant_fp8(x); wq,sw=K.quant_weight_fp8(w)
    tf=t(lambda: K.gemm_fp8(xq,sa,wq,sw))
    tq=t(lambda: K.quant_fp8(x, out=xq, scale=sa))
    tt=t(lambda: torch._scaled_mm(xq, wq.t(), scale_a=sa.view(-1,1), scale_b=sw.view(1,-1), out_dtype=torch.bfloat16)) if hasattr(torch,'_scaled_mm') else float('nan')
    print(f"M={M} N={N} K={Kd} bf16={fl/tb/1e9:.0f}TF fp8={fl/tf/1e9:.0f}TF quant={tq*1e3:.0f}us fp8+quant={fl/(tf+tq)/1e9:.0f}TF torch_scaled_mm={fl/tt/1e9:.0f}TF", flush=True)
PY
timeout -k 10 300 python - <<'PY'
import torch, sys, time
sys.path.insert(0, '.')
from docagents_amd.models.bert import BertEncoder
from docagents_amd.models.configs import encoder_config
for arch in ("bge-base", "bge-large"):
    cfg = encoder_config(arch)
    a = BertEncoder(cfg, "cuda", seed=1)
    b = BertEncoder(cfg, "cuda", weights=a.w, dtype="fp8")
    seqs = [[101] + [1000 + (i * 7 + j) % 20000 for j in range(510)] + [102] for i in range(128)]
    res = {}
    for name, enc in (("bf16", a), ("fp8", b)):
        for _ in range(2): enc.encode_packed(seqs)
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(5): v = enc.encode_packed(seqs)
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 5
        res[name] = (dt, v)
    cos = (res["bf16"][1] * res["fp8"][1]).sum(-1)
    tok = 128 * 512
    print(f"{arch}: bf16 {tok/res['bf16'][0]:.0f} tok/s  fp8 {tok/res['fp8'][0]:.0f} tok/s  speedup {res['bf16'][0]/res['fp8'][0]:.2f}x  min cos {cos.min().item():.4f}", flush=True)
PY
