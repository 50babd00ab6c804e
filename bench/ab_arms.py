"""A/B arms for the microbenchmarks — NOT part of the production ops.

The production GEMM entry point (``docagents_amd.ops.kernels.gemm``) only dispatches to the in-tree
gfx950 kernels. What round 1-2 kept behind ``DA_BLAS_*`` / ``DA_*`` switches inside that module
lives here now, for comparisons only:

* ``blas_gemm`` / ``blas_swiglu``: the platform BLAS (hipBLASLt through ``torch.mm``) for the same
  products, so ``bench/gemm_ab.py`` can time gemm8p against the vendor library on one box;
* ``swiglu_interleaved``: the standalone SwiGLU pass the BLAS arm needs (the in-tree GEMM fuses it);
* ``apply_env_overrides``: kernel-schedule overrides (decode-tile prefetch depth, flash prefill
  shape, GEMV blocking, decode-attention prefetch) read from ``DA_*`` environment variables and
  pushed into the library's setters, and the model's alternative code paths (fused prefill norms,
  the persistent batch-1 decode), so a sweep can flip one knob per process. ``bench.py`` applies
  them too (nothing happens without a ``DA_*`` variable set).
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402

ENV_SETTERS = {
    "DA_GEMM_PF": "da_set_gemm_pf",          # decode-tile k-tiles in flight
    "DA_DK_RB": "da_set_dk_rb",              # gemm_dk 33..64 rows: two 32-row blocks (1) / one 64-row block (0)
    "DA_GEMM_DB": "da_set_gemm_db",          # decode tiles load W fragments straight to registers
    "DA_DECODE_BALANCE": "da_set_decode_balance",  # decode attention: balanced vs fixed keys per split
    "DA_DECODE_QFIRST": "da_set_decode_qfirst",    # batch-1 decode attention: prologue loads before K/V
    "DA_FLASH_PIPE": "da_set_flash_pipe",    # software-pipelined flash prefill on / off / auto
    "DA_FLASH_QH": "da_set_flash_qh",        # flash queries per wave: 1 = 32, 2 = 64
    "DA_FLASH_WAVES": "da_set_flash_waves",  # flash waves per workgroup
    "DA_FLASH_REV": "da_set_flash_rev",      # flash dispatch: bit 0 causal longest-first, bit 1 XCD-grouped
    "DA_GEMV_U": "da_set_gemv_u",            # batch-1 GEMV K-blocks in flight per row
    "DA_GEMV_KS": "da_set_gemv_ks",          # batch-1 GEMV waves per long row
    "DA_DECODE_PFT": "da_set_decode_pft",    # MHA decode next-tile prefetch threshold
    "DA_DECODE_W8": "da_set_decode_w8",      # ... with 8 waves per workgroup up to this many (row, kv head) pairs
    "DA_DECODE_W8_VAR": "da_set_decode_w8_var",  # ... 0: two tiles per wave (spills), 1: one tile per wave
    "DA_GEMM8P_GROUP": "da_set_gemm8p_group",  # prefill GEMM tile-order band height (0 = auto)
    "DA_GEMM8P_BM_RULE": "da_set_gemm8p_bm_rule",  # prefill row-tile height: 1 = fewest waves, 0 = round-3 rule
    "DA_OMERGE_SHAPE": "da_set_omerge_shape",  # merged batch-1 O GEMV: waves per workgroup * 10 + rows per wave
}


def apply_env_overrides() -> dict:
    """Push every DA_* schedule override present in the environment into the library."""
    L = K.lib()
    done = {}
    from docagents_amd.models import llama
    for env, attr in (("DA_PREFILL_NORM_FUSE", "_PREFILL_NORM_FUSE"), ("DA_DECODE_B1", "_DECODE_B1"),
                      ("DA_O_MERGE", "_O_MERGE"), ("DA_QKV_FOLD", "_QKV_FOLD")):
        if os.environ.get(env) is not None:  # model-level code paths (default: llama.py)
            setattr(llama, attr, os.environ[env] == "1")
            done[env] = int(getattr(llama, attr))
    if os.environ.get("DA_SPLITK_FUSED") is not None:  # 33..64-row decode: in-kernel split-K reduce
        from docagents_amd.ops import reference as R
        K.SPLITK_FUSED = R.SPLITK_FUSED = os.environ["DA_SPLITK_FUSED"] != "0"
        done["DA_SPLITK_FUSED"] = int(K.SPLITK_FUSED)
    if os.environ.get("DA_DECODE_DK") is not None:  # decode GEMMs: gemm_dk (1) vs split-K tiles (0)
        K.DECODE_DK = os.environ["DA_DECODE_DK"] != "0"
        done["DA_DECODE_DK"] = int(K.DECODE_DK)
    for env, fn in ENV_SETTERS.items():
        v = os.environ.get(env)
        if v is not None:
            getattr(L, fn)(int(v))
            done[env] = int(v)
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
