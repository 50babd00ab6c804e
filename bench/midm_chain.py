"""Mid-M GEMMs (decode batches 65..1023, short prefills): a 32-layer Phi-3 projection chain (qkv, o,
gate/up + SwiGLU, down; 7.2 GB of bf16 weights, far beyond the Infinity Cache) captured in one HIP
graph and replayed, in-tree tiles vs hipBLASLt. Arms: "blas", "auto" (the production route) or
"tile:splits" (tile 2 = 64x128 decode tile over ceil(M/64) row blocks, 7 / 10 = phase-split 256- /
128-row tiles, 8 = 128x128 PF4, 9 = 128x64 PF4; splits 0 = the auto split rule)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import apply_env_overrides, swiglu_interleaved  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps (DA_GEMM_DB, DA_GEMM_PF, ...)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--ms", default="80,128,256,512,1000")
    ap.add_argument("--arms", default="blas,auto,2:1,2:2,2:4,10:1")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H, I = 3072, 8192
    shapes = [(3 * H, H), (H, H), (2 * I, H), (H, I)]
    g = torch.Generator(device=dev).manual_seed(0)
    W = [[(torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16) for n, k in shapes]
         for _ in range(a.layers)]
    gb = sum(w.numel() * 2 for L in W for w in L) / 1e9
    for M in [int(m) for m in a.ms.split(",")]:
        x = torch.randn(M, I, device=dev).to(torch.bfloat16)
        outs = [torch.empty(M, n, device=dev, dtype=torch.bfloat16) for n, _ in shapes]
        act = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        K.reserve_workspace(8 * M * 2 * I * 4, dev)
        res = {}
        for arm in a.arms.split(","):
            def run():
                for L in W:
                    for j, w in enumerate(L):
                        xi = x[:, :w.shape[1]]
                        if arm == "blas":
                            torch.matmul(xi, w.t(), out=outs[j])
                            if j == 2:
                                swiglu_interleaved(outs[j], act)
                        elif arm == "auto":  # the production route (K.gemm defaults)
                            if j == 2:
                                K.gemm(xi, w, epi=K.EPI_SWIGLU, out=act)
                            else:
                                K.gemm(xi, w, out=outs[j])
                        else:
                            t, s = (int(v) for v in arm.split(":"))
                            if s == 0:
                                s = K._auto_splits(max(M, 1), w.shape[0], w.shape[1])
                            if j == 2:
                                K.gemm(xi, w, epi=K.EPI_SWIGLU, out=act, tile=t, splits=s)
                            else:
                                K.gemm(xi, w, out=outs[j], tile=t, splits=s)
            try:
                run(); torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                res[arm] = str(e)[:60]
                continue
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                run()
            graph.replay(); torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                graph.replay()
            e.record(); torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 5
            res[arm] = round(ms, 3)
            del graph
        best = min((v, k) for k, v in res.items() if isinstance(v, float))
        print(json.dumps({"M": M, "ms": res, "best": best[1], "best_TBps": round(gb / best[0], 2)}), flush=True)


if __name__ == "__main__":
    main()
