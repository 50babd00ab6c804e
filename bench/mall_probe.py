"""Does a batch-1 GEMV run faster when its weights were read shortly before (Infinity Cache / MALL
hit) than from HBM? Per Phi-3 decode weight (O 3072x3072, QKV 9216x3072, gate/up 16384x3072,
down 3072x8192): the GEMV time (events, median of REPS) after a 1 GiB flush read, after the flush
plus a plain read of the weight (torch.sum), and back to back (second of two GEMVs). One JSON line
per weight. Decides whether prefetching the next projection's weights beside a latency-bound kernel
(the batch-1 decode attention) can pay."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", "20"))
    dev = torch.device("cuda")
    flush = torch.ones(1 << 29, dtype=torch.bfloat16, device=dev)  # 1 GiB
    shapes = {"o": (3072, 3072, K.EPI_RESID), "qkv": (9216, 3072, K.EPI_NONE),
              "gate_up": (16384, 3072, K.EPI_SWIGLU), "down": (3072, 8192, K.EPI_RESID)}
    for name, (N, Kd, epi) in shapes.items():
        w = (torch.randn((N, Kd), device=dev) * 0.02).to(torch.bfloat16)
        x = torch.randn((1, Kd), device=dev).to(torch.bfloat16)
        r = torch.randn((1, N), device=dev).to(torch.bfloat16) if epi == K.EPI_RESID else None

        def run():
            return K.gemm(x, w, epi=epi, resid=r)

        res = {}
        for arm in ("cold", "prefetched", "back_to_back"):
            ts = []
            for _ in range(reps):
                flush.sum()
                if arm == "prefetched":
                    w.sum()
                if arm == "back_to_back":
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000)
            res[arm] = round(statistics.median(ts), 2)
        mb = N * Kd * 2 / 1e6
        print(json.dumps({"weight": name, "MB": round(mb, 1), "us": res,
                          "TBps": {k: round(mb / v, 2) for k, v in res.items()}}), flush=True)  # MB/us = TB/s


if __name__ == "__main__":
    main()
