"""64-row decode GEMMs on the 64x128 split-K tiles + reduce, per Phi-3 shape, over a range of split
counts (not only powers of two), 32 distinct HBM-resident weights captured in one graph; us per
GEMM. Picks the split the 33..64-row route should use."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H, I, L, M = 3072, 8192, 32, int(os.environ.get("M", "64"))
    shapes = {"qkv": (3 * H, H, K.EPI_NONE), "o": (H, H, K.EPI_RESID), "gateup": (2 * I, H, K.EPI_SWIGLU),
              "down": (H, I, K.EPI_RESID)}
    g = torch.Generator(device=dev).manual_seed(0)
    res = {"M": M}
    for name, (N, Kd, epi) in shapes.items():
        W = [(torch.randn(N, Kd, device=dev, generator=g) * 0.02).bfloat16() for _ in range(L)]
        x = torch.randn(M, Kd, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16() if epi == K.EPI_RESID else None
        out = torch.empty(M, N // 2 if epi == K.EPI_SWIGLU else N, device=dev, dtype=torch.bfloat16)
        K.reserve_workspace(16 * M * N * 4, dev)
        row = {}
        for s in (2, 3, 4, 6, 8, 12, 16):
            if (Kd // 64) % s or (N // 128) * s > 400:
                continue
            def run():
                for w in W:
                    K.gemm(x, w, epi=epi, resid=r, out=out, tile=2, splits=s)
            run(); torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                run()
            gr.replay(); torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                gr.replay()
            b.record(); torch.cuda.synchronize()
            row[s] = round(a.elapsed_time(b) / 10 / L * 1e3, 2)
            del gr
        res[name] = row
        del W
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
