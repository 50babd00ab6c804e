"""Batch-1 prefill projections (M ~ 2.6k suffix tokens of the p50 query) on 256- vs 128-row tiles of
the phase-split GEMM, 32 distinct weight sets per shape (the layer sequence: weights not
cache-warm), graph-replayed; us per GEMM. One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    torch.manual_seed(0)
    M = int(os.environ.get("M", "2632"))
    for N, Kd, epi in [(3072, 3072, K.EPI_RESID), (3072, 8192, K.EPI_RESID), (9216, 3072, K.EPI_NONE),
                       (16384, 3072, K.EPI_SWIGLU)]:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        ws = [((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16() for _ in range(32)]
        nout = N // 2 if epi == K.EPI_SWIGLU else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        resid = torch.zeros(M, nout, device="cuda", dtype=torch.bfloat16) if epi == K.EPI_RESID else None
        res = {"M": M, "N": N, "K": Kd, "epi": epi}
        outs = {}
        for rnd in range(3):
            for tile in (7, 10):
                def run():
                    for w in ws:
                        K.gemm(x, w, epi=epi, resid=resid, out=out, tile=tile, splits=1)
                run()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    run()
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    g.replay()
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1000 / 5 / len(ws)
                key = f"bm{256 if tile == 7 else 128}_us"
                res[key] = min(res.get(key, 1e9), round(us, 2))
                outs[tile] = out.clone()
        res["same_bits"] = bool(torch.equal(outs[7], outs[10]))
        K.lib().da_set_gemm8p_bm_rule(1)
        print(json.dumps(res), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
