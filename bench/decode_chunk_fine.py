"""Decode attention at small batch: fine chunk sweep (multiples of 64 keys) with the in-kernel split
merge, graph-style max_len = cache capacity (the split count a captured decode graph uses)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def t(fn, it=100):
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


for (B, L) in [(1, 2944), (1, 1500), (2, 2944), (4, 2944), (8, 2944)]:
    H = Hkv = 32
    D, S = 96, 4096
    kc = torch.randn(B, Hkv, S, D, device='cuda').bfloat16()
    vc = torch.randn_like(kc)
    q = torch.randn(B, (H + 2 * Hkv) * D, device='cuda').bfloat16()
    lens = torch.full((B,), L, device='cuda', dtype=torch.int32)
    slot = torch.arange(B, device='cuda', dtype=torch.int32)
    by = 2 * B * Hkv * L * D * 2
    out = []
    for ch in (192, 256, 320, 384, 448, 512, 640, 768, 1024):
        tt = t(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S, chunk=ch))
        out.append(f"c{ch}={tt * 1e3:.1f}")
    ta = t(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S))
    print(f"B={B} L={L}: " + " ".join(out) + f" auto={ta * 1e3:.1f}us ({by / ta / 1e9:.2f} TB/s)", flush=True)
