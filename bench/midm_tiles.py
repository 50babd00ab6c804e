"""Mid-M (65..128-row) decode GEMM tiles, cold weights, per Phi-3 shape: tile x splits sweep plus a
numerics check of every arm against tile 2 (the production route's tile for N >= 8192).
  python bench/midm_tiles.py [--m 128] [--arms 2:1,9:1,11:1,13:1,...]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from decode_gemm_sweep import timed  # noqa: E402

SHAPES = [("qkv", 9216, 3072, K.EPI_NONE), ("o", 3072, 3072, K.EPI_NONE), ("gu", 16384, 3072, K.EPI_SWIGLU),
          ("down", 3072, 8192, K.EPI_NONE), ("lm", 32064, 3072, K.EPI_NONE)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=128)
    ap.add_argument("--arms", default="0:0,2:1,2:2,9:1,9:4,8:1,8:2")
    a = ap.parse_args()
    M = a.m
    for name, N, Kd, epi in SHAPES:
        x = torch.randn(M, Kd, device="cuda").bfloat16()
        by = N * Kd * 2
        ncopy = max(2, (1 << 30) // by + 1)
        ws = [(torch.randn(N, Kd, device="cuda") * 0.02).bfloat16() for _ in range(ncopy)]
        nout = N // 2 if epi == K.EPI_SWIGLU else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        ref = K.gemm(x, ws[0], epi=epi, tile=2, splits=1).float()
        res = {}
        for arm in a.arms.split(","):
            t, s = (int(v) for v in arm.split(":"))
            if N % 64 and t in (9, 11):
                continue
            K.reserve_workspace(max(1, s) * M * N * 4 + (1 << 20), torch.device("cuda"))
            try:
                got = K.gemm(x, ws[0], epi=epi, tile=t, splits=s).float()
                err = float((got - ref).abs().max())
                us = timed(lambda i: K.gemm(x, ws[i % ncopy], epi=epi, out=out, tile=t, splits=s), 2 * ncopy)
                res[arm] = {"us": round(us, 2), "TBps": round(by / us / 1e6, 2), "maxdiff": round(err, 4)}
            except Exception as e:  # noqa: BLE001
                res[arm] = {"error": repr(e)[:80]}
        best = min((k for k in res if "us" in res[k]), key=lambda k: res[k]["us"])
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": Kd, "best": best, "arms": res}), flush=True)


if __name__ == "__main__":
    main()
