"""How much of a prefill GEMM is per-tile fixed cost (prologue fill + epilogue stores) rather than
K-loop: time the phase-split GEMM at one (M, N) for several K and fit t = a K + e (e = the per-launch
fixed part, which scales with the tile count, not with K)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    M = 65536
    for N, epi in ((9216, K.EPI_NONE), (16384, K.EPI_SWIGLU), (3072, K.EPI_NONE)):
        pts = []
        for Kd in (1024, 2048, 3072, 4096, 6144):
            a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, Kd, device=dev) * Kd ** -0.5).to(torch.bfloat16)
            out = torch.empty(M, N // 2 if epi == K.EPI_SWIGLU else N, device=dev, dtype=torch.bfloat16)
            ms = timed(lambda: K.gemm(a, w, epi=epi, out=out))
            pts.append((Kd, ms))
            del a, w, out
        n = len(pts)
        mx = sum(k for k, _ in pts) / n
        my = sum(t for _, t in pts) / n
        slope = sum((k - mx) * (t - my) for k, t in pts) / sum((k - mx) ** 2 for k, _ in pts)
        icpt = my - slope * mx
        t3072 = dict(pts)[3072]
        print(json.dumps({"M": M, "N": N, "epi": epi, "ms_by_K": {k: round(t, 4) for k, t in pts},
                          "fixed_ms": round(icpt, 4), "fixed_share_at_K3072": round(icpt / t3072, 3),
                          "tflops_at_K3072": round(2 * M * N * 3072 / t3072 / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
