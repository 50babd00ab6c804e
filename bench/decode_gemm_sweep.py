"""Decode GEMMs (M <= 128): split-K LDS tile (--tiles to compare tiles), register prefetch depth PF x split count. Timed the way the decoder runs them: one HIP graph of
back-to-back calls, each on a different weight copy (>= 1 GiB of copies, so every call streams its
weights cold from HBM as a decode step does). Times include the split-K reduction / fused epilogue
exactly as the decoder calls it (o / down: resid + RMSNorm tail; gate/up: SwiGLU; qkv / LM head:
plain).

  python bench/decode_gemm_sweep.py [--shapes phi3|llama8b|all]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

SHAPES = {
    "phi3": [("qkv", 9216, 3072, "plain"), ("o", 3072, 3072, "norm"), ("gu", 16384, 3072, "swiglu"),
             ("down", 3072, 8192, "norm"), ("lm", 32064, 3072, "plain")],
    "llama8b": [("qkv", 6144, 4096, "plain"), ("o", 4096, 4096, "norm"), ("gu", 28672, 4096, "swiglu"),
                ("down", 4096, 14336, "norm"), ("lm", 128256, 4096, "plain")],
}


def timed(run, n, reps=5):
    """us per call: graph of n calls (call i on weight copy i), replayed reps times."""
    for i in range(n):
        run(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            run(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) / (reps * n) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="phi3")
    ap.add_argument("--m", default="64,16")
    ap.add_argument("--tiles", default="auto", help="comma list of gemm tiles (2 = 64x128, 9 = 128x64, ...) or auto")
    a = ap.parse_args()
    models = list(SHAPES) if a.shapes == "all" else a.shapes.split(",")
    for model in models:
        for M in [int(x) for x in a.m.split(",")]:
            for name, N, Kd, kind in SHAPES[model]:
                x = torch.randn(M, Kd, device="cuda").bfloat16()
                by = N * Kd * 2
                ncopy = max(2, (1 << 30) // by + 1)
                ws = [(torch.randn(N, Kd, device="cuda") * Kd ** -0.5).bfloat16() for _ in range(ncopy)]
                resid = torch.randn(M, N, device="cuda").bfloat16()
                gamma = torch.ones(N, device="cuda").bfloat16()

                def runner(tile, splits):
                    def run(i):
                        if kind == "norm":
                            K.gemm_resid_norm(x, ws[i], resid, gamma, 1e-5, out=resid, tile=tile, splits=splits)
                        else:
                            K.gemm(x, ws[i], epi=K.EPI_SWIGLU if kind == "swiglu" else K.EPI_NONE, tile=tile,
                                   splits=splits)
                    return run
                res = {}
                auto_s = K._auto_splits(M, N, Kd)
                tiles = [K._decode_tile(M)] if a.tiles == "auto" else [int(t) for t in a.tiles.split(",")]
                for tile in tiles:
                    if kind == "norm" and M > 64 and tile != 9:
                        continue  # the fused reduce + norm runs on the 128x64 tile above 64 rows
                    for sp in (1, 2, 4, 8, 16):
                        if (Kd // 64) % sp:
                            continue
                        res[f"t{tile}s{sp}" if len(tiles) > 1 else f"s{sp}"] = timed(runner(tile, sp), ncopy)
                best = min(res, key=res.get)
                print(json.dumps({"model": model, "gemm": name, "M": M, "N": N, "K": Kd, "MB": round(by / 1e6, 1),
                                  "us": {k: round(v, 1) for k, v in res.items()}, "auto_splits": auto_s,
                                  "best": best, "best_TBps": round(by / res[best] / 1e6, 2)}), flush=True)
                del ws


if __name__ == "__main__":
    main()
