"""Dense-scan probe: time the streaming top-k kernels (ops.kernels.topk_dense's route) on one shard
for several batch sizes, similarity floors (a floor no row passes = pure streaming, no candidate
work) and rows per wave, to separate HBM streaming from the top-K bookkeeping."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--qs", default="1,16,17,32,64")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, d = a.rows, a.dim
    X = torch.empty(N, d, device=dev, dtype=torch.bfloat16)
    for s in range(0, N, 1 << 20):  # normalised random rows, built in slices
        e = min(N, s + (1 << 20))
        X[s:e] = torch.nn.functional.normalize(torch.randn(e - s, d, device=dev), dim=-1).to(torch.bfloat16)
    gb = N * d * 2 / 1e9
    lib = K.lib()
    for q in [int(x) for x in a.qs.split(",")]:
        Qv = torch.nn.functional.normalize(torch.randn(q, d, device=dev), dim=-1).to(torch.bfloat16)
        base = max(64, math.ceil(N / (256 * 16) / 16) * 16)
        for thr in (-1.0, 0.95):
            for rpw in (base, base * 4):
                ws = K._workspace(int(lib.da_topk_stream_ws(N, q, a.k, rpw)), dev)
                out_s = torch.empty((q, a.k), dtype=torch.float32, device=dev)
                out_i = torch.empty((q, a.k), dtype=torch.int32, device=dev)

                def run():
                    K._check(lib.da_topk_dense_stream(K._ptr(X), N, d, None, K._ptr(Qv), q, None, 0, float(thr), a.k,
                                                      rpw, K._ptr(ws), K._ptr(out_s), K._ptr(out_i), K._stream()), "scan")
                run(); torch.cuda.synchronize()
                s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                for _ in range(a.reps):
                    run()
                e0.record(); torch.cuda.synchronize()
                ms = s0.elapsed_time(e0) / a.reps
                print(json.dumps({"Q": q, "thr": thr, "rows_per_wave": rpw, "ms": round(ms, 3),
                                  "TBps": round(gb / ms, 2)}), flush=True)


if __name__ == "__main__":
    main()
