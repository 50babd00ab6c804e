"""Prefill GEMM A/B: persistent tile loop (one workgroup per CU) vs one workgroup per tile, on the
Phi-3-mini prefill products at a QA chunk (M = 65536) and at the batch-1 prefill (M = 2600); the
two modes alternate over 3 rounds in one process (K.gemm8p_persist), median of each."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402


def timed(fn, reps=15):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[reps // 2]


def cases(M, dev, g):
    Kd = 3072
    a = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(9216, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    c = torch.empty(M, 9216, device=dev, dtype=torch.bfloat16)
    H = Hkv = 32
    D, L = 96, 2048
    pos = (torch.arange(M, device=dev, dtype=torch.int32) % L)
    slot = (torch.arange(M, device=dev, dtype=torch.int32) // L)
    S = int(slot.max()) + 1
    cs = R.rope_table(L, D, 10000.0, device=dev)
    kc = torch.empty(S, Hkv, L, D, device=dev, dtype=torch.bfloat16)
    vc = torch.empty_like(kc)
    w2 = (torch.randn(3072, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    x = torch.randn(M, 3072, device=dev, generator=g).to(torch.bfloat16)
    c2 = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
    w3 = (torch.randn(16384, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    c3 = torch.empty(M, 8192, device=dev, dtype=torch.bfloat16)
    a4 = torch.randn(M, 8192, device=dev, generator=g).to(torch.bfloat16)
    w4 = (torch.randn(3072, 8192, device=dev, generator=g) * 8192 ** -0.5).to(torch.bfloat16)
    return {
        f"rope_qkv_{M}": (lambda: K.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc, vc, out=c, kv_out=False),
                          2 * M * 9216 * Kd),
        f"o_resid_{M}": (lambda: K.gemm(a, w2, epi=K.EPI_RESID, resid=x, out=c2), 2 * M * 3072 * Kd),
        f"gate_up_swiglu_{M}": (lambda: K.gemm(a, w3, epi=K.EPI_SWIGLU, out=c3), 2 * M * 16384 * Kd),
        f"down_resid_{M}": (lambda: K.gemm(a4, w4, epi=K.EPI_RESID, resid=x, out=c2), 2 * M * 3072 * 8192),
    }


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    prev = K.gemm8p_persist(-1)
    try:
        for M in (65536, 2600):
            cs_ = cases(M, dev, g)
            for name, (fn, flops) in cs_.items():
                t = {0: [], 1: []}
                for _ in range(3):
                    for mode in (0, 1):
                        K.gemm8p_persist(mode)
                        t[mode].append(timed(fn))
                off, on = statistics.median(t[0]), statistics.median(t[1])
                res[name] = {"per_tile_ms": round(off, 4), "persistent_ms": round(on, 4),
                             "speedup": round(off / on, 4), "persistent_tflops": round(flops / on / 1e9, 1)}
                print(json.dumps({name: res[name]}), flush=True)
            del cs_
            torch.cuda.empty_cache()
    finally:
        K.gemm8p_persist(prev)
    print(json.dumps({"summary": res}), flush=True)


if __name__ == "__main__":
    main()
