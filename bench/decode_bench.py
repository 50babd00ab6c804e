"""Decode-path microbenchmarks on MI355X: decode attention variants, RoPE+cache write, skinny GEMMs."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps


def timeit(fn, iters=20):
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
    for name, B, L, H, Hkv, D in [("phi3_b64", 64, 2944, 32, 32, 96), ("llama3_b64", 64, 4096, 32, 8, 128),
                                  ("phi3_b32", 32, 2944, 32, 32, 96),
                                  ("llama70b_tp8_b64", 64, 4096, 8, 1, 128), ("llama3_b16_short", 16, 512, 32, 8, 128),
                                  ("gqa2_d64", 32, 2048, 8, 4, 64)]:
        S = L + 64
        kc = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16)
        q = torch.randn(B, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        lens = torch.full((B,), L, device=dev, dtype=torch.int32)
        slot = torch.arange(B, device=dev, dtype=torch.int32)
        by = 2 * B * Hkv * L * D * 2
        r = {}
        t = timeit(lambda: K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S))
        r["ours"] = dict(ms=t, tbps=by / t / 1e9)
        res[f"decode_attn/{name}"] = r
        print(name, json.dumps(r), flush=True)
    # rope + cache write at decode size
    for T in (64, 4096):
        H, Hkv, D = 32, 32, 96
        qkv = torch.randn(T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        kc = torch.zeros(65, Hkv, 4096, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
        slot = torch.randint(0, 64, (T,), device=dev, dtype=torch.int32)
        cs = R.rope_table(4096, D, 10000.0).to(dev)
        t = timeit(lambda: K.rope_cache(qkv, pos, cs, H, Hkv, D, slot=slot, k_cache=kc, v_cache=vc))
        res[f"rope_cache/T{T}"] = dict(us=t * 1e3)
        print("rope", T, t * 1e3, "us", flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
