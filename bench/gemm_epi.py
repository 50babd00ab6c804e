"""Epilogue cost of the prefill GEMM (gemm8p) at the Phi-3 QA prefill-chunk shapes (M = 57344 rows):
each projection with its production epilogue (QKV + RoPE + KV-cache write, O / down + residual,
gate/up + SwiGLU) vs the same product with the plain epilogue, randn * 0.02 weights like the model.
Prints ms and TF/s per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def timeit(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("M", "57344"))
    H, I, D = 3072, 8192, 96
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, I, device=dev, generator=g).bfloat16()
    res = {}
    # QKV: plain vs RoPE + cache
    w = (torch.randn(3 * H, H, device=dev, generator=g) * 0.02).bfloat16()
    out = torch.empty(M, 3 * H, device=dev, dtype=torch.bfloat16)
    a = x[:, :H]
    cs = torch.randn(8192, D // 2, 2, device=dev)
    kc = torch.empty(24, 32, 8192, D, device=dev, dtype=torch.bfloat16)
    vc = torch.empty_like(kc)
    pos = (torch.arange(M, device=dev, dtype=torch.int32) % 2930)
    slot = (torch.arange(M, device=dev, dtype=torch.int32) // 2930)
    fl = 2 * M * 3 * H * H
    t0 = timeit(lambda: K.gemm(a, w, out=out))
    t1 = timeit(lambda: K.gemm_rope(a, w, pos, cs, 32, 32, D, slot, kc, vc, out=out))
    res["qkv"] = {"plain_ms": round(t0, 3), "rope_ms": round(t1, 3), "plain_TF": round(fl / t0 / 1e9), "rope_TF": round(fl / t1 / 1e9)}
    # O: plain vs residual
    w = (torch.randn(H, H, device=dev, generator=g) * 0.02).bfloat16()
    out = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
    r = torch.randn(M, H, device=dev, generator=g).bfloat16()
    fl = 2 * M * H * H
    t0 = timeit(lambda: K.gemm(a, w, out=out))
    t1 = timeit(lambda: K.gemm(a, w, epi=K.EPI_RESID, resid=r, out=out))
    res["o"] = {"plain_ms": round(t0, 3), "resid_ms": round(t1, 3), "plain_TF": round(fl / t0 / 1e9), "resid_TF": round(fl / t1 / 1e9)}
    # gate/up: plain (N = 16384 out) vs SwiGLU (N/2 out)
    w = (torch.randn(2 * I, H, device=dev, generator=g) * 0.02).bfloat16()
    out = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * 2 * I * H
    t0 = timeit(lambda: K.gemm(a, w, out=out))
    t1 = timeit(lambda: K.gemm(a, w, epi=K.EPI_SWIGLU, out=out[:, :I]))
    res["gateup"] = {"plain_ms": round(t0, 3), "swiglu_ms": round(t1, 3), "plain_TF": round(fl / t0 / 1e9), "swiglu_TF": round(fl / t1 / 1e9)}
    # down: plain vs residual
    w = (torch.randn(H, I, device=dev, generator=g) * 0.02).bfloat16()
    out = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * H * I
    t0 = timeit(lambda: K.gemm(x, w, out=out))
    t1 = timeit(lambda: K.gemm(x, w, epi=K.EPI_RESID, resid=r, out=out))
    res["down"] = {"plain_ms": round(t0, 3), "resid_ms": round(t1, 3), "plain_TF": round(fl / t0 / 1e9), "resid_TF": round(fl / t1 / 1e9)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
