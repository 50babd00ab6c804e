"""Compute ops: hand-written gfx950 HIP kernels (``kernels``) and their fp32 PyTorch oracles
(``reference``). ``get_ops(device)`` returns the kernel module for GPU tensors and the reference
module for CPU tensors — never a silent fallback on a GPU device."""
from __future__ import annotations

import torch


def get_ops(device):
    dev = torch.device(device)
    if dev.type == "cuda":
        from . import kernels
        kernels.lib()  # fail loudly if the HIP library is missing
        return kernels
    from . import reference
    return reference
