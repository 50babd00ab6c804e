"""Prefill attention microbenchmark: the production flash dispatch (ops.flash_attn_varlen: the pipelined
causal D = 96 kernel, flash_attn_v2 otherwise) vs torch SDPA on MI355X shapes, checked against SDPA."""
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
    for name, B, L, H, Hkv, D, causal in [("phi3_qa_chunk", 22, 2938, 32, 32, 96, True),
                                          ("phi3_prefill", 8, 2944, 32, 32, 96, True),
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
        t = timeit(lambda: K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal))
        out = K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal).float()
        r["ours"] = {"ms": round(t, 3), "tflops": round(fl / t / 1e9, 1),
                     "max_err_vs_sdpa": round((out - ref).abs().max().item(), 4)}
        t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal))
        r["sdpa"] = {"ms": round(t, 3), "tflops": round(fl / t / 1e9, 1)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
