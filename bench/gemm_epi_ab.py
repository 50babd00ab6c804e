"""Prefill GEMM epilogue A/B: the phase-split GEMM's four prefill epilogues at a QA chunk (M = 65536,
K = 3072; RoPE: Phi-3 heads, k / v to the cache only) timed with the kernel library given by
DA_LIB (default: the in-tree one). Run once per library, alternating."""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

if os.environ.get("DA_LIB"):
    import ctypes
    K._LIB_PATH = Path(os.environ["DA_LIB"])
    _probe = ctypes.CDLL(str(K._LIB_PATH))  # an older library lacks newer exports: do not bind those
    K._SIGS = {n: a for n, a in K._SIGS.items() if hasattr(_probe, n)}


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    M, Kd = 65536, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    out = {}
    w = (torch.randn(9216, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    c = torch.empty(M, 9216, device=dev, dtype=torch.bfloat16)
    out["none_9216"] = timed(lambda: K.gemm(a, w, out=c))
    H = Hkv = 32
    D, S, L = 96, 32, 2048
    pos = (torch.arange(M, device=dev, dtype=torch.int32) % L)
    slot = (torch.arange(M, device=dev, dtype=torch.int32) // L)
    cs = R.rope_table(L, D, 10000.0, device=dev)
    kc = torch.empty(S, Hkv, L, D, device=dev, dtype=torch.bfloat16)
    vc = torch.empty_like(kc)
    out["rope_9216"] = timed(lambda: K.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc, vc, out=c, kv_out=False))
    w2 = (torch.randn(3072, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    x = torch.randn(M, 3072, device=dev, generator=g).to(torch.bfloat16)
    c2 = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
    out["resid_3072"] = timed(lambda: K.gemm(a, w2, epi=K.EPI_RESID, resid=x, out=c2))
    out["none_3072"] = timed(lambda: K.gemm(a, w2, out=c2))
    w3 = (torch.randn(16384, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    c3 = torch.empty(M, 8192, device=dev, dtype=torch.bfloat16)
    out["swiglu_16384"] = timed(lambda: K.gemm(a, w3, epi=K.EPI_SWIGLU, out=c3))
    print(json.dumps({"lib": os.environ.get("DA_LIB", "in-tree"), "persist": os.environ.get("DA_GEMM8P_PERSIST", "default"), "ms": {k: round(v, 4) for k, v in out.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
