"""Decode attention: split-KV chunk size sweep at small and large batch (sets the auto-chunk rule),
with the in-kernel split merge (fused) and the separate combine launch (unfused)."""
import sys

import torch

sys.path.insert(0, '.')
from docagents_amd.ops import kernels as K  # noqa: E402


def t(fn, it=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for (B, H, Hkv, D, L) in [(1, 32, 32, 96, 2944), (4, 32, 32, 96, 2944), (1, 32, 8, 128, 2944),
                          (16, 32, 32, 96, 2944), (64, 32, 32, 96, 2944)]:
    S = 4096
    kc = torch.randn(B, Hkv, S, D, device='cuda').bfloat16()
    vc = torch.randn_like(kc)
    q = torch.randn(B, (H + 2 * Hkv) * D, device='cuda').bfloat16()
    lens = torch.full((B,), L, device='cuda', dtype=torch.int32)
    slot = torch.arange(B, device='cuda', dtype=torch.int32)
    by = 2 * B * Hkv * L * D * 2
    for fused in (False, True):
        K._FUSED_COMBINE = fused
        out = []
        for ch in (64, 128, 256, 512, 1024, 2048, 4096):
            tt = t(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S, chunk=ch))
            out.append(f"c{ch}={tt * 1e3:.1f}us")
        ta = t(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S))
        print(f"B={B} H={H} Hkv={Hkv} D={D} L={L} fused={int(fused)}: " + " ".join(out)
              + f" auto={ta * 1e3:.1f}us ({by / ta / 1e9:.2f} TB/s)", flush=True)
