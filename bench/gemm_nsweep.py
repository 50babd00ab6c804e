"""Prefill GEMM (gemm8p, plain epilogue) TF/s vs N at M = 57344, K = 3072, each shape timed twice
in interleaved order (clock warm-up / ordering effects show as a spread between the two)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def timeit(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


dev = torch.device("cuda")
M = int(os.environ.get("M", "57344"))
Kd = int(os.environ.get("KD", "3072"))
Ns = [int(v) for v in os.environ.get("NS", "3072,8192,9216,10240,16384").split(",")]
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
W = {n: (torch.randn(n, Kd, device=dev, generator=g) * 0.02).bfloat16() for n in Ns}
out = torch.empty(M, max(Ns), device=dev, dtype=torch.bfloat16)
res = {n: [] for n in Ns}
for rnd in range(2):
    for n in (Ns if rnd == 0 else Ns[::-1]):
        o = out[:, :n]
        t = timeit(lambda: K.gemm(x, W[n], out=o))
        res[n].append(round(2 * M * n * Kd / t / 1e9))
print(json.dumps({"M": M, "K": Kd, "TFps": res}), flush=True)
