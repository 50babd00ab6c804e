"""One prefill-attention shape, repeated (for rocprofv3 PMC passes): phi3 (causal, D=96; phi3qa = the
QA prefill chunk, 22 x 2938) or bge (D=64)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

SHAPES = {"phi3": (8, 2944, 32, 32, 96, True), "phi3qa": (22, 2938, 32, 32, 96, True), "bge": (64, 512, 12, 12, 64, False)}
B, L, H, Hkv, D, causal = SHAPES[os.environ.get("SHAPE", "phi3")]
dev = torch.device("cuda")
torch.manual_seed(0)
T = B * L
qkv = torch.randn(T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
cu = torch.arange(0, T + 1, L, device=dev, dtype=torch.int32)
for _ in range(int(os.environ.get("REPS", "5"))):
    K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal)
torch.cuda.synchronize()
