"""Prefill attention microbenchmark: flash_attn_v2 (4- and 8-wave workgroups) vs torch SDPA on MI355X shapes."""
import argparse
import os
import sys
import json

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.ops import kernels as K  # noqa: E402


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
        for impl in ("v2", "v2w8"):
            K.lib().da_set_flash_waves(8 if impl == "v2w8" else 4)
            t = timeit(lambda: K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal))
            r[impl + "_ms"], r[impl + "_tflops"] = t, fl / t / 1e9
        K.lib().da_set_flash_waves(8)
        o8 = K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal).float()
        K.lib().da_set_flash_waves(0)
        qq = q.reshape(B, L, H, D).transpose(1, 2)
        kk = k.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        vv = v.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal))
        r["sdpa_ms"], r["sdpa_tflops"] = t, fl / t / 1e9
        o1 = K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal).float()
        o2 = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal)
        o2 = o2.transpose(1, 2).reshape(T, H * D).float()
        r["max_err_vs_sdpa"] = (o1 - o2).abs().max().item()
        r["w8_vs_w4_maxdiff"] = (o8 - o1).abs().max().item()
        res[name] = r
        print(name, json.dumps(r), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
