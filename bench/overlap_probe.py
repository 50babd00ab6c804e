"""Probe: does memory-bound decode attention overlap with compute-bound prefill GEMMs when the two
run on separate HIP streams of one MI355X?  (Decides whether the serving loop should co-schedule
one batch's decode with the next batch's prefill.)

Prints the wall time of (a) decode attention alone, (b) prefill GEMMs alone, (c) both issued
concurrently on two streams, and the overlap efficiency  (a + b - c) / min(a, b).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ctx", type=int, default=2934)
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--attn-iters", type=int, default=96)
    ap.add_argument("--gemm-iters", type=int, default=12)
    ap.add_argument("--gemm", default="own", choices=["own", "torch"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    H = Hkv = 32
    D = 96
    S = a.batch
    cap = (a.ctx + 255) // 256 * 256
    kc = torch.randn((S, Hkv, cap, D), device=dev).to(torch.bfloat16)
    vc = torch.randn((S, Hkv, cap, D), device=dev).to(torch.bfloat16)
    q = torch.randn((S, H * D), device=dev).to(torch.bfloat16)
    lens = torch.full((S,), a.ctx, dtype=torch.int32, device=dev)
    slot = torch.arange(S, dtype=torch.int32, device=dev)
    out = torch.empty((S, H * D), dtype=torch.bfloat16, device=dev)
    x = torch.randn((a.m, 3072), device=dev).to(torch.bfloat16)
    w = (torch.randn((16384, 3072), device=dev) * 0.02).to(torch.bfloat16)
    y = torch.empty((a.m, 16384), dtype=torch.bfloat16, device=dev)
    ysw = torch.empty((a.m, 8192), dtype=torch.bfloat16, device=dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def attn():
        with torch.cuda.stream(sa):
            for _ in range(a.attn_iters):
                K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, cap, out=out)

    def gemm():
        with torch.cuda.stream(sb):
            for _ in range(a.gemm_iters):
                if a.gemm == "torch":
                    torch.matmul(x, w.t(), out=y)
                else:
                    K.gemm(x, w, epi=K.EPI_SWIGLU, out=ysw)  # gemm256 + fused SwiGLU (the MLP up-proj)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1000

    for _ in range(2):
        timed(attn); timed(gemm); timed(lambda: (attn(), gemm()))
    ta = min(timed(attn) for _ in range(3))
    tg = min(timed(gemm) for _ in range(3))
    tc = min(timed(lambda: (gemm(), attn())) for _ in range(3))
    kv_bytes = 2 * S * Hkv * a.ctx * D * 2 * a.attn_iters
    flops = 2 * a.m * 3072 * 16384 * a.gemm_iters
    res = {"attn_ms": round(ta, 2), "gemm_ms": round(tg, 2), "concurrent_ms": round(tc, 2),
           "serial_ms": round(ta + tg, 2), "overlap_eff": round((ta + tg - tc) / min(ta, tg), 3),
           "attn_TBps": round(kv_bytes / ta / 1e9, 2), "gemm_TFps": round(flops / tg / 1e9, 1), "gemm": a.gemm}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
