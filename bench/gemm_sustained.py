"""Sustained (power-capped) GEMM throughput: ours (gemm256) vs hipBLASLt (torch.matmul) on the
prefill projection shapes, each run back-to-back for ~SECS seconds so the clock settles at the
level the flagship bench sees (short bursts over-report: MI355X_MICROARCH 'DVFS give-back')."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps

SECS = float(os.environ.get("SECS", "2"))
only = os.environ.get("ONLY", "")


def run(fn, flop):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    burst = None
    while True:
        for _ in range(4):
            fn()
        n += 4
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if burst is None:
            burst = flop * n / el / 1e12
        if el > SECS:
            break
    # last 25 % of the window: settled clock
    t1 = time.perf_counter()
    m = max(4, n // 4)
    for _ in range(m):
        fn()
    torch.cuda.synchronize()
    return burst, flop * m / (time.perf_counter() - t1) / 1e12


for (M, N, Kd) in [(32768, 9216, 3072), (32768, 16384, 3072), (32768, 3072, 8192), (32768, 3072, 3072)]:
    x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    flop = 2 * M * N * Kd
    res = []
    arms = {"ours": lambda: K.gemm(x, w, tile=4, splits=1, out=out),
            "ours_pp": None,
            "ours_w4": lambda: K.gemm(x, w, tile=5, splits=1, out=out),
            "ours_w4s5": None,
            "ours_w4m1": None,
            "ours_w4m1s5": None,
            "diag_nodma": None,
            "ours_w4m3": None,
            "diag_dma0": None,
            "hipblaslt": lambda: torch.matmul(x, w.t(), out=out)}
    for name, fn in arms.items():
        if only and name not in only.split(","):
            continue
        if (name.startswith("ours_w4") and name != "ours_w4") or name.startswith("diag"):
            K.lib().da_set_gemm_w4_cfg({"ours_w4s5": 1, "ours_w4m1": 2, "ours_w4m1s5": 3, "diag_nodma": 4, "ours_w4m3": 5, "diag_dma0": 6}[name])
            b, s = run(lambda: K.gemm(x, w, tile=5, splits=1, out=out), flop)
            K.lib().da_set_gemm_w4_cfg(0)
        elif name == "ours_pp":
            K.lib().da_set_gemm_pingpong(1)
            b, s = run(lambda: K.gemm(x, w, tile=4, splits=1, out=out), flop)
            K.lib().da_set_gemm_pingpong(0)
        else:
            b, s = run(fn, flop)
        res.append(f"{name}: burst {b:.0f} sustained {s:.0f}")
    print(f"M={M} N={N} K={Kd}: " + "; ".join(res), flush=True)
