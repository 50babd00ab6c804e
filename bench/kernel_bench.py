"""Micro-benchmarks of the gfx950 kernels against PyTorch-ROCm (hipBLASLt / SDPA) on the shapes the
flagship pipeline runs (Phi-3-mini QA, BGE-base encoder, 100k-row flat index).

python bench/kernel_bench.py [--out profiles/kernel_bench.json]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    res = {}
    torch.manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev) * scale).to(torch.bfloat16)

    gemms = [("phi3_qkv_prefill", 4096, 9216, 3072), ("phi3_gateup_prefill", 4096, 16384, 3072),
             ("phi3_down_prefill", 4096, 3072, 8192), ("bge_ffn1", 8192, 3072, 768),
             ("phi3_qkv_decode_b32", 32, 9216, 3072), ("phi3_gateup_decode_b64", 64, 16384, 3072),
             ("phi3_down_decode_b64", 64, 3072, 8192), ("phi3_lmhead_b64", 64, 32064, 3072)]
    for name, M, N, Kd in gemms:
        x, w = rnd(M, Kd), rnd(N, Kd, scale=Kd ** -0.5)
        t_ours = timeit(lambda: K.gemm(x, w))
        t_torch = timeit(lambda: torch.matmul(x, w.t()))
        fl = 2 * M * N * Kd
        by = 2 * (M * Kd + N * Kd + M * N)
        res[f"gemm/{name}"] = dict(M=M, N=N, K=Kd, ours_ms=t_ours, torch_ms=t_torch,
                                   ours_tflops=fl / t_ours / 1e9, torch_tflops=fl / t_torch / 1e9,
                                   ours_gbps=by / t_ours / 1e6, torch_gbps=by / t_torch / 1e6)
        print(name, res[f"gemm/{name}"], flush=True)
    # swiglu fused vs separate
    M, F, Kd = 4096, 8192, 3072
    x, w = rnd(M, Kd), rnd(2 * F, Kd, scale=Kd ** -0.5)
    t = timeit(lambda: K.gemm(x, w, epi=K.EPI_SWIGLU))
    res["gemm/phi3_gateup_swiglu_fused"] = dict(ours_ms=t, ours_tflops=2 * M * 2 * F * Kd / t / 1e9)
    print("swiglu", res["gemm/phi3_gateup_swiglu_fused"], flush=True)

    # attention prefill (Phi-3: H=32, D=96 causal; BGE: H=12, D=64 bidirectional)
    for name, B, L, H, Hkv, D, causal in [("phi3_prefill", 8, 2944, 32, 32, 96, True),
                                          ("bge_base", 64, 512, 12, 12, 64, False),
                                          ("llama3_prefill", 4, 4096, 32, 8, 128, True)]:
        T = B * L
        qkv = rnd(T, (H + 2 * Hkv) * D)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
        cu = torch.arange(0, T + 1, L, device=dev, dtype=torch.int32)
        t_ours = timeit(lambda: K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal), iters=5)
        qq = q.reshape(B, L, H, D).transpose(1, 2)
        kk = k.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        vv = v.reshape(B, L, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, 1)
        t_torch = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal),
                         iters=5)
        fl = 4 * B * L * L * H * D * (0.5 if causal else 1.0)
        res[f"attn/{name}"] = dict(ours_ms=t_ours, torch_sdpa_ms=t_torch, ours_tflops=fl / t_ours / 1e9,
                                   torch_tflops=fl / t_torch / 1e9)
        print(name, res[f"attn/{name}"], flush=True)

    # decode attention: bandwidth
    for name, B, L, H, Hkv, D in [("phi3_decode_b32", 32, 2944, 32, 32, 96), ("llama3_decode_b64", 64, 4096, 32, 8, 128)]:
        kc, vc = rnd(B, Hkv, L, D), rnd(B, Hkv, L, D)
        q = rnd(B, (H + 2 * Hkv) * D)
        lens = torch.full((B,), L, device=dev, dtype=torch.int32)
        slot = torch.arange(B, device=dev, dtype=torch.int32)
        t = timeit(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=L))
        by = 2 * B * Hkv * L * D * 2
        res[f"decode_attn/{name}"] = dict(ms=t, gbps=by / t / 1e6)
        print(name, res[f"decode_attn/{name}"], flush=True)

    # flat index scan
    for N, d, Q in [(100_000, 768, 64), (1_000_000, 768, 16)]:
        X = torch.nn.functional.normalize(torch.randn(N, d, device=dev), dim=-1).to(torch.bfloat16)
        Qv = torch.nn.functional.normalize(torch.randn(Q, d, device=dev), dim=-1).to(torch.bfloat16)
        t = timeit(lambda: K.topk_dense(X, Qv, 5, -1.0))
        t_torch = timeit(lambda: torch.topk((Qv @ X.t()).float(), 5, dim=1))
        res[f"topk_dense/N{N}_Q{Q}"] = dict(ms=t, torch_ms=t_torch, gbps=N * d * 2 * math.ceil(Q / 16) / t / 1e6)
        print(N, Q, res[f"topk_dense/N{N}_Q{Q}"], flush=True)

    # norms
    x = rnd(8192, 3072); w = rnd(3072); r = rnd(8192, 3072)
    t = timeit(lambda: K.rmsnorm(x, w, 1e-5, resid=r))
    res["rmsnorm/8192x3072_resid"] = dict(ms=t, gbps=8192 * 3072 * 2 * 4 / t / 1e6)
    logits = rnd(64, 32064, scale=3)
    t = timeit(lambda: K.sample(logits, 0.2, 1, 2))
    res["sample/64x32064"] = dict(ms=t)
    print(res, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
