"""Decode GEMMs at 33..64 rows, per Phi-3 layer shape (qkv, o + residual, gate/up + SwiGLU, down +
residual), each over 32 distinct weight matrices captured in one graph (HBM-resident, like the
decode chain): the split-K tiles + reduce ("splitk") vs gemm_dk (two 32-row blocks per n-tile).
Prints us per GEMM and TB/s of weight bytes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H, I, L = 3072, 8192, 32
    shapes = {"qkv": (3 * H, H, K.EPI_NONE), "o": (H, H, K.EPI_RESID), "gateup": (2 * I, H, K.EPI_SWIGLU),
              "down": (H, I, K.EPI_RESID)}
    g = torch.Generator(device=dev).manual_seed(0)
    for M in [int(m) for m in os.environ.get("MS", "64,40").split(",")]:
        res = {"M": M}
        for name, (N, Kd, epi) in shapes.items():
            W = [(torch.randn(N, Kd, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(L)]
            x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
            r = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == K.EPI_RESID else None
            nout = N // 2 if epi == K.EPI_SWIGLU else N
            out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
            K.reserve_workspace(8 * M * N * 4, dev)
            row = {}
            for arm in ("splitk", "dk"):
                def run():
                    for w in W:
                        if arm == "splitk":
                            K.gemm(x, w, epi=epi, resid=r, out=out, tile=2 if M > 32 else 3, splits=0)
                        else:
                            K.gemm_dk(x, w, epi=epi, resid=r, out=out)
                run(); torch.cuda.synchronize()
                ref = out.clone()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    run()
                graph.replay(); torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    graph.replay()
                e.record(); torch.cuda.synchronize()
                us = s.elapsed_time(e) / 10 / L * 1e3
                row[arm] = {"us": round(us, 2), "TBps": round(N * Kd * 2 / us / 1e6, 2)}
                if arm == "splitk":
                    base = ref
                else:
                    row[arm]["maxdiff_vs_splitk"] = round((ref.float() - base.float()).abs().max().item(), 4)
                del graph
            res[name] = row
            del W
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
