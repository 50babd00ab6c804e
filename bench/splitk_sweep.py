"""Decode-sized (M = 64) GEMM: tile x split-K sweep (sets _auto_splits)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for name, M, N, Kd, epi in [("qkv", 64, 9216, 3072, 0), ("o", 64, 3072, 3072, 4), ("gu", 64, 16384, 3072, 3),
                            ("down", 64, 3072, 8192, 4), ("lm", 64, 32064, 3072, 0), ("qkv_b16", 16, 9216, 3072, 0),
                            ("down_b16", 16, 3072, 8192, 4)]:
    x = torch.randn(M, Kd, device="cuda").bfloat16()
    w = (torch.randn(N, Kd, device="cuda") * Kd ** -0.5).bfloat16()
    r = torch.randn(M, N, device="cuda").bfloat16() if epi == 4 else None
    by = N * Kd * 2
    out = [f"auto(s={K._auto_splits(M, N, Kd)})={t(lambda: K.gemm(x, w, epi=epi, resid=r)) * 1e3:.1f}"]
    for tile in (2, 3):
        for s in (1, 2, 4, 8, 16, 32):
            if (Kd // 64) % s:
                continue
            us = t(lambda: K.gemm(x, w, epi=epi, resid=r, tile=tile, splits=s)) * 1e3
            out.append(f"t{tile}s{s}={us:.1f}")
    print(f"{name} M={M} N={N} K={Kd} ({by / 1e6:.0f} MB): " + " ".join(out), flush=True)
