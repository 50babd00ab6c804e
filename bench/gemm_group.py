"""Prefill GEMM (gemm8p, 256x256 tiles) vs the grouped-M band height of its tile order
(da_set_gemm8p_group; GRP="2,4" picks the arms): Phi-3 prefill shapes, interleaved rounds, sustained TF/s on random
[-1, 1) operands. One JSON line per shape."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

GROUPS = [int(g) for g in os.environ.get("GRP", "1,2,4,8,16").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", "3"))


def rate(fn, flop, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return flop * reps / (s.elapsed_time(e) / 1000) / 1e12


def main():
    torch.manual_seed(0)
    shapes = [(65536, 9216, 3072, K.EPI_NONE), (65536, 16384, 3072, K.EPI_SWIGLU), (65536, 3072, 3072, K.EPI_RESID),
              (65536, 3072, 8192, K.EPI_RESID), (29440, 9216, 3072, K.EPI_NONE)]
    for M, N, Kd, epi in shapes:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
        nout = N // 2 if epi == K.EPI_SWIGLU else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        resid = torch.zeros(M, nout, device="cuda", dtype=torch.bfloat16) if epi == K.EPI_RESID else None
        flop = 2.0 * M * N * Kd
        res = {"shape": [M, N, Kd, epi]}
        ref = None
        for _ in range(ROUNDS):
            for g in GROUPS:
                K.lib().da_set_gemm8p_group(g)
                fn = lambda: K.gemm(x, w, epi=epi, resid=resid, out=out, tile=7, splits=1)  # noqa: E731
                tf = rate(fn, flop)
                res[f"g{g}"] = max(res.get(f"g{g}", 0.0), round(tf, 1))
                if ref is None:
                    ref = out.clone()
                else:
                    assert torch.equal(out, ref), "tile order changed the result"
        K.lib().da_set_gemm8p_group(0)
        print(json.dumps(res), flush=True)
        del x, w, out, resid
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
