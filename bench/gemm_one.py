"""One prefill-shaped GEMM repeated (for rocprofv3 counter collection).

python bench/gemm_one.py [M N K]; env ARM = tile id of the in-tree kernel (default 7 = gemm8p) or "blas"."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps

M, N, Kd = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32768, 9216, 3072)))
arm = os.environ.get("ARM", "7")
x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
tile = arm
for _ in range(5):
    if arm == "blas":
        torch.mm(x, w.t(), out=out)
    else:
        K.gemm(x, w, tile=int(tile), splits=1, out=out)
torch.cuda.synchronize()
print("ok")
