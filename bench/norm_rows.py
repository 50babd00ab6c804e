"""Prefill-chunk RMSNorm bandwidth: M rows of D (the QA prefill's 57k x 3072), with and without the
fused residual add; bytes moved / time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda")
res = {}
for M, D in ((57344, 3072), (16384, 4096), (1023, 3072)):
    x = torch.randn(M, D, device=dev).bfloat16()
    w = torch.randn(D, device=dev).bfloat16()
    y = torch.empty_like(x)
    r = torch.randn(M, D, device=dev).bfloat16()
    for tag, fn, nbytes in (("norm", lambda: K.rmsnorm(x, w, 1e-5, out=y), 2 * M * D * 2),
                            ("resid_norm", lambda: K.rmsnorm(x, w, 1e-5, resid=r, out=y), 4 * M * D * 2)):
        fn(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record(); torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        res[f"{M}x{D}_{tag}"] = {"us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}
print(json.dumps(res), flush=True)
