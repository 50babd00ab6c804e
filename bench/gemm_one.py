"""One prefill-shaped GEMM repeated (for rocprofv3 counter collection)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

M, N, Kd = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32768, 9216, 3072)))
x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * Kd ** -0.5).bfloat16()
for _ in range(5):
    K.gemm(x, w, tile=int(os.environ.get("TILE", "4")), splits=1)
torch.cuda.synchronize()
print("ok")
