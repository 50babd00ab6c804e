"""Decode-sized (M = 64) GEMM: tile x split-K sweep (sets _auto_splits). Weights are cycled through
enough copies (>= 1 GiB) that every call streams them cold from HBM, as in a real decode step
(each layer's weights are read once per step; 7.6 GB/step for Phi-3 >> the 256 MB MALL)."""
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
                            ("down_b16", 16, 3072, 8192, 4), ("qkv_b1", 1, 9216, 3072, 0), ("gu_b1", 1, 16384, 3072, 3),
                            ("down_b1", 1, 3072, 8192, 4)]:
    x = torch.randn(M, Kd, device="cuda").bfloat16()
    by = N * Kd * 2
    ncopy = max(2, (1 << 30) // by + 1)
    ws = [(torch.randn(N, Kd, device="cuda") * Kd ** -0.5).bfloat16() for _ in range(ncopy)]
    r = torch.randn(M, N, device="cuda").bfloat16() if epi == 4 else None
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % ncopy
        return ws[it[0]]
    out = [f"auto(s={K._auto_splits(M, N, Kd)})={t(lambda: K.gemm(x, nxt(), epi=epi, resid=r)) * 1e3:.1f}"]
    for tile in (2, 3):
        for s in (1, 2, 4, 8, 16, 32):
            if (Kd // 64) % s:
                continue
            us = t(lambda: K.gemm(x, nxt(), epi=epi, resid=r, tile=tile, splits=s)) * 1e3
            out.append(f"t{tile}s{s}={us:.1f}")
    if M == 1:
        out.append(f"gemv={t(lambda: K.gemm(x, nxt(), epi=epi, resid=r, tile=6, splits=1)) * 1e3:.1f}")
    print(f"{name} M={M} N={N} K={Kd} ({by / 1e6:.0f} MB, cold): " + " ".join(out), flush=True)
    del ws
