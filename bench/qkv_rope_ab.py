"""Prefill QKV projection + attention at a QA chunk (22 prompts x 2944 tokens, Phi-3: 32 heads,
D = 96): the k / v written to the KV cache AND the qkv tile with the attention reading the tile
(kv_out=1, round 4), vs the cache only with the attention reading the cache (kv_out=0, round 5).
usage: qkv_rope_ab.py [--arm 0|1|both] [--reps N]; under scripts/gpu_pmc.sh give one arm."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", default="both")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--seqs", type=int, default=22)
    ap.add_argument("--len", type=int, default=2944)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H = Hkv = 32
    D, hid, S = 96, 3072, a.len + 128
    T = a.seqs * a.len
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(T, hid, device=dev, generator=g)).to(torch.bfloat16)
    w = (torch.randn((H + 2 * Hkv) * D, hid, device=dev, generator=g) * hid ** -0.5).to(torch.bfloat16)
    slot = torch.arange(T, device=dev, dtype=torch.int32) // a.len
    pos = torch.arange(T, device=dev, dtype=torch.int32) % a.len
    cu = torch.arange(0, T + 1, a.len, device=dev, dtype=torch.int32)
    cs = R.rope_table(S, D, 10000.0, device=dev)
    kc = torch.zeros(a.seqs, Hkv, S, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    qkv = torch.empty(T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    out = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)

    def gemm(kv_out):
        K.gemm_rope(x, w, pos, cs, H, Hkv, D, slot, kc, vc, out=qkv, kv_out=bool(kv_out))

    def attn(kv_out):
        if kv_out:
            K.flash_attn_varlen(qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:], cu, a.len,
                                H, Hkv, D, True, out=out)
        else:
            K.flash_attn_varlen(qkv[:, :H * D], None, None, cu, a.len, H, Hkv, D, True, out=out,
                                kv_cache=(kc, vc, slot, pos))

    arms = [0, 1] if a.arm == "both" else [int(a.arm)]
    gflop = 2 * T * hid * (H + 2 * Hkv) * D / 1e9
    aflop = 2 * 2 * H * D * a.seqs * a.len * (a.len + 1) / 2 / 1e9  # causal
    res = {arm: {"gemm_ms": [], "attn_ms": []} for arm in arms}
    for arm in arms:  # warm
        gemm(arm); attn(arm)
    torch.cuda.synchronize()
    for _ in range(a.reps):  # interleaved arms
        for arm in arms:
            for name, fn in (("gemm_ms", gemm), ("attn_ms", attn)):
                s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record(); fn(arm); e0.record(); torch.cuda.synchronize()
                res[arm][name].append(s0.elapsed_time(e0))
    for arm in arms:
        gm = sorted(res[arm]["gemm_ms"])[len(res[arm]["gemm_ms"]) // 2]
        am = sorted(res[arm]["attn_ms"])[len(res[arm]["attn_ms"]) // 2]
        print(json.dumps({"kv_out": arm, "tokens": T, "gemm_ms_median": round(gm, 4),
                          "gemm_tflops": round(gflop / gm, 1), "attn_ms_median": round(am, 4),
                          "attn_tflops": round(aflop / am, 1)}), flush=True)


if __name__ == "__main__":
    main()
