"""gemm4w (four-wave 256x256, csrc/gemm4w.hip) schedule variants vs gemm8p (tile 7) vs hipBLASLt.

python bench/gemm4w_ab.py [arms] — arms: "7", "blas", "13:<v>" (v = kernels.gemm4w_variant:
0 three fragment sets + two barriers per K-tile, 1 two sets, 2 three sets + one barrier). Checks every 13:* arm against an fp32 reference first, then prints sustained TF/s per shape (interleaved
rounds, random operands)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import blas_gemm  # noqa: E402
from gemm_ab import rate  # noqa: E402

ARMS = (sys.argv[1] if len(sys.argv) > 1 else "7,13:0,13:1,13:2,blas").split(",")
ROUNDS = int(os.environ.get("ROUNDS", "3"))
SHAPES = [(32768, 9216, 3072), (32768, 3072, 8192), (32768, 3072, 3072), (8192, 8192, 8192), (2930, 9216, 3072)]


def call(arm, x, w, out):
    if arm == "blas":
        return blas_gemm(x, w, epi=K.EPI_NONE, out=out)
    if arm.startswith("13:"):
        K.gemm4w_variant(int(arm[3:]))
        return K.gemm(x, w, out=out, tile=13, splits=1)
    return K.gemm(x, w, out=out, tile=int(arm), splits=1)


def main():
    torch.manual_seed(0)
    for (M, N, Kd) in [(1000, 1000, 128), (777, 2048, 1024), (5000, 9216, 3072)]:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
        ref = x.float() @ w.float().t()
        for arm in ARMS:
            if not arm.startswith("13:"):
                continue
            out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            call(arm, x, w, out)
            err = (out.float() - ref).abs().max().item()
            if not err <= 0.02 + 0.01 * ref.abs().max().item():
                print(json.dumps({"check": [M, N, Kd], "arm": arm, "max_err": err, "ok": False}), flush=True)
                sys.exit(1)
    only = os.environ.get("SHAPES")
    shapes = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for (M, N, Kd) in shapes:
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {a: [] for a in ARMS}
        for _ in range(ROUNDS):
            for a in ARMS:
                res[a].append(round(rate(lambda: call(a, x, w, out), 2 * M * N * Kd), 1))
        print(json.dumps({"shape": [M, N, Kd], **{a: max(v) for a, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
