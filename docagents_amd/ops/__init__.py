"""Compute ops: hand-written gfx950 HIP kernels (``kernels``) and their fp32 PyTorch oracles
(``reference``). ``get_ops(device)`` returns the kernel module for GPU tensors and the reference
module for CPU tensors — never a silent fallback on a GPU device."""
from __future__ import annotations

import numpy as np
import torch


def h2d(a, dev) -> torch.Tensor:
    """Host array -> device tensor without blocking the host: the array is staged in PyTorch's
    cached pinned-host allocator (which records the copy's stream, so the block is not reused
    before the copy ran). A pageable-memory copy would make the host wait for the current stream
    to drain first, which serialises work the host issues to several streams (the search plane,
    the fast embed lane and the decode thread each run on a stream of their own)."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    dev = torch.device(dev)
    if dev.type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def get_ops(device):
    dev = torch.device(device)
    if dev.type == "cuda":
        from . import kernels
        kernels.lib()  # fail loudly if the HIP library is missing
        return kernels
    from . import reference
    return reference
