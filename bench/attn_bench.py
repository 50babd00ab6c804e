"""Prefill attention microbenchmark: flash_attn_v2 arms (4 / 8 waves per workgroup x 32 / 64 queries per wave)
vs torch SDPA on MI355X shapes, each arm checked against SDPA."""
import argparse
import os
import sys
import json

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    res = {}
    for name, B, L, H, Hkv, D, causal in [("phi3_prefill", 8, 2944, 32, 32, 96, True),
                                          ("bge_base", 64, 512, 12, 12, 64, False),
                                          ("bge_small", 64, 512, 12, 12, 32, False),
                                          ("llama3_prefill", 4, 4096, 32, 8, 128, True),
                                          ("bge_large", 64, 512, 16, 16, 64, False)]:
        T = B * L
        qkv = torch.randn(T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
        cu = torch.arange(0, T + 1, L, device=dev, dtype=torch.int32)
        fl = 4 * B * L * L * H * D * (0.5 if causal else 1.0)
        r = {}
        qq = q.reshape(B, L, H, D).transpose(1, 2)
        kk = k.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        vv = v.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        ref = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal)
        ref = ref.transpose(1, 2).reshape(T, H * D).float()
        # arms: waves per workgroup x 32-query halves per wave
        for nw, qh, pipe in ((4, 1, 0), (8, 1, 0), (4, 2, 0), (8, 2, 0), (4, 1, 1), (4, 1, 3), (4, 1, 4)):
            if (nw * qh > 8 and D > 64) or (pipe and D > 96):
                continue
            K.lib().da_set_flash_waves(nw)
            K.lib().da_set_flash_qh(qh)
            K.lib().da_set_flash_pipe(pipe)
            arm = f"w{nw}q{qh}" + ("", "pipe", "", "spec", "dma")[pipe]
            t = timeit(lambda: K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal))
            out = K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal).float()
            r[arm] = {"ms": round(t, 3), "tflops": round(fl / t / 1e9, 1),
                      "max_err_vs_sdpa": round((out - ref).abs().max().item(), 4)}
        K.lib().da_set_flash_waves(0)
        K.lib().da_set_flash_qh(0)
        K.lib().da_set_flash_pipe(K.FLASH_PIPE_DEFAULT)
        t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal))
        r["sdpa"] = {"ms": round(t, 3), "tflops": round(fl / t / 1e9, 1)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
