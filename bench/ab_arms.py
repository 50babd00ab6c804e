"""A/B arms for the microbenchmarks — NOT part of the production ops.

The production GEMM entry point (``docagents_amd.ops.kernels.gemm``) only dispatches to the in-tree
gfx950 kernels. What round 1-2 kept behind ``DA_BLAS_*`` / ``DA_*`` switches inside that module
lives here now, for comparisons only:

* ``blas_gemm`` / ``blas_swiglu``: the platform BLAS (hipBLASLt through ``torch.mm``) for the same
  products, so ``bench/gemm_ab.py`` can time gemm8p against the vendor library on one box;
* ``swiglu_interleaved``: the standalone SwiGLU pass the BLAS arm needs (the in-tree GEMM fuses it);
* ``apply_env_overrides``: the model-level decode GEMM route read from ``DA_DECODE_DK``, so a
  sweep can flip it per process. ``bench.py`` applies it too (nothing happens without it set).
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

def apply_env_overrides() -> dict:
    """Model-level switches read from ``DA_*`` environment variables (one per process):
    DA_DECODE_DK=0 routes 2..64-row decode GEMMs to the split-K tiles instead of gemm_dk. The kernel
    schedule setters and the rejected decode / prefill arms of rounds 1-4 were removed from the
    library (git history keeps them; profiles/r4/rejected_r4.txt has their numbers)."""
    done = {}
    if os.environ.get("DA_DECODE_DK") is not None:  # decode GEMMs: gemm_dk (1) vs split-K tiles (0)
        K.DECODE_DK = os.environ["DA_DECODE_DK"] != "0"
        done["DA_DECODE_DK"] = int(K.DECODE_DK)
    return done


def swiglu_interleaved(x: torch.Tensor, out=None) -> torch.Tensor:
    """[M, 2F] gate/up (16-column interleave, the EPI_SWIGLU weight order) -> silu(gate) * up [M, F]."""
    K._bf16_cuda(x, "x")
    M, N2 = x.shape
    K._req(N2 % 32 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0, "x must be [M, 2F] row-major, F % 16 == 0")
    if out is None:
        out = torch.empty((M, N2 // 2), dtype=torch.bfloat16, device=x.device)
    K._check(K.lib().da_swiglu_interleaved(K._ptr(x), x.stride(0), K._ptr(out), out.stride(0), M, N2 // 2,
                                           K._stream()), "swiglu_interleaved")
    return out


def blas_gemm(a, w, bias=None, epi: int = K.EPI_NONE, resid=None, out=None) -> torch.Tensor:
    """The vendor-library arm of gemm(): plain / bias / residual (beta = 1) products."""
    wt = w.t()
    if epi == K.EPI_SWIGLU:
        return swiglu_interleaved(torch.mm(a, wt), out)
    if epi == K.EPI_NONE:
        return torch.mm(a, wt, out=out)
    if epi == K.EPI_BIAS:
        return torch.addmm(bias, a, wt, out=out)
    if epi != K.EPI_RESID or bias is not None:
        raise ValueError("blas_gemm: NONE / BIAS / RESID (no bias) / SWIGLU only")
    if out is not None and out.data_ptr() == resid.data_ptr() and out.stride() == resid.stride():
        return out.addmm_(a, wt)
    return torch.addmm(resid, a, wt, out=out)
