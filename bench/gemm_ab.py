"""Prefill GEMM A/B: in-tree 256x256 kernels vs hipBLASLt, correctness first, then sustained TF/s.

Usage: python bench/gemm_ab.py [arms] — arms is a comma list of tile ids / "blas" (default
"4,7,blas"). Every arm runs on the same random [-1, 1) operands, interleaved over ROUNDS rounds in
one process (cdna_hip_programming.md §5.4 rules 24/25); prints one JSON line per shape.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import blas_gemm  # noqa: E402

ARMS = (sys.argv[1] if len(sys.argv) > 1 else "4,7,blas").split(",")
SECS = float(os.environ.get("SECS", "0.5"))
ROUNDS = int(os.environ.get("ROUNDS", "3"))
EPI = {"none": K.EPI_NONE, "swiglu": K.EPI_SWIGLU, "resid": K.EPI_RESID, "gelu": K.EPI_GELU, "bias": K.EPI_BIAS}


def call(arm, x, w, out, epi, bias=None, resid=None):
    if arm == "blas":
        return blas_gemm(x, w, epi=epi if epi in (K.EPI_SWIGLU, K.EPI_NONE) else K.EPI_NONE, out=out)
    tile = arm
    return K.gemm(x, w, bias=bias, epi=epi, resid=resid, out=out, tile=int(tile), splits=1)


def check():
    torch.manual_seed(0)
    bad = 0
    for (M, N, Kd, epi) in [(1000, 1000, 128, "none"), (300, 520, 192, "bias"), (4096, 3072, 3072, "none"),
                            (2900, 768, 768, "gelu"), (1024, 4096, 640, "swiglu"), (777, 2048, 1024, "resid"),
                            (256, 256, 64 * 3, "none"), (5000, 9216, 3072, "none")]:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
        bias = (torch.rand(N, device="cuda") - 0.5).bfloat16() if epi in ("bias", "gelu", "resid") else None
        resid = (torch.rand(M, N, device="cuda") - 0.5).bfloat16() if epi == "resid" else None
        ref = x.float() @ w.float().t()
        if bias is not None:
            ref = ref + bias.float()
        if epi == "gelu":
            ref = torch.nn.functional.gelu(ref)
        if epi == "resid":
            ref = ref + resid.float()
        if epi == "swiglu":
            r = ref.view(M, N // 32, 2, 16)
            ref = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(M, N // 2)
        for arm in ARMS:
            if arm == "blas":
                continue
            out = torch.full(ref.shape, float("nan"), device="cuda", dtype=torch.bfloat16)
            call(arm, x, w, out, EPI[epi], bias, resid)
            torch.cuda.synchronize()
            err = (out.float() - ref).abs().max().item()
            tol = 0.02 + 0.01 * ref.abs().max().item()
            ok = err <= tol and not torch.isnan(out).any().item()
            bad += not ok
            print(json.dumps({"check": [M, N, Kd, epi], "arm": arm, "max_err": round(err, 5), "tol": round(tol, 4),
                              "ok": ok}), flush=True)
    return bad


def rate(fn, flop):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < SECS:
        for _ in range(4):
            fn()
        n += 4
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    m = max(4, n // 2)
    for _ in range(m):
        fn()
    torch.cuda.synchronize()
    return flop * m / (time.perf_counter() - t1) / 1e12


def perf():
    shapes = [(32768, 9216, 3072, "none"), (32768, 16384, 3072, "swiglu"), (32768, 3072, 8192, "none"),
              (32768, 3072, 3072, "none"), (8192, 8192, 8192, "none"), (29440, 9216, 3072, "none"),
              (65536, 768, 3072, "none"), (65536, 3072, 768, "none"),
              # batch-1 prefill (~2.9k tokens): 256-row tiles underfill the chip at N = 3072
              (2930, 3072, 3072, "none"), (2930, 3072, 8192, "none"), (2930, 9216, 3072, "none"),
              (2930, 16384, 3072, "swiglu"), (512, 9216, 3072, "none"), (256, 9216, 3072, "none"),
              # batch-1 prefill after the kept 256-token prompt head (~2.6k suffix tokens)
              (2614, 3072, 3072, "resid"), (2614, 3072, 8192, "resid"), (2614, 9216, 3072, "none"),
              (2614, 16384, 3072, "swiglu")]
    only = os.environ.get("SHAPES")
    if only:
        shapes = [shapes[int(i)] for i in only.split(",")]
    for (M, N, Kd, epi) in shapes:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
        out = torch.empty(M, N // 2 if epi == "swiglu" else N, device="cuda", dtype=torch.bfloat16)
        flop = 2 * M * N * Kd
        resid = (torch.rand(M, N, device="cuda") - 0.5).bfloat16() if epi == "resid" else None
        res = {a: [] for a in ARMS}
        for _ in range(ROUNDS):
            for a in ARMS:
                res[a].append(round(rate(lambda: call(a, x, w, out, EPI[epi], resid=resid), flop), 1))
        print(json.dumps({"shape": [M, N, Kd, epi], **{a: max(v) for a, v in res.items()},
                          "rounds": res}), flush=True)


if __name__ == "__main__":
    nbad = check()
    if nbad:
        print(f"{nbad} correctness failures", flush=True)
        sys.exit(1)
    perf()
