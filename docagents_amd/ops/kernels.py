"""ctypes bindings for the gfx950 kernel library (``_da_kernels.so``).

Every wrapper validates shapes / dtypes / contiguity / device on the host BEFORE launching (a
mis-shaped launch of a hand-written kernel can fault the GPU), launches on PyTorch's current HIP
stream, and raises on any launch error. There is deliberately no silent fallback: on a GPU box,
if the library is missing the import fails loudly (``KernelLibraryMissing``). The fp32 PyTorch
oracles for tests live in ``docagents_amd.ops.reference``.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
import threading
from pathlib import Path

import torch

_LIB = None
_LOCK = threading.Lock()
# DA_KERNELS_DEBUG=1: the -DDA_DEBUG build (device asserts: bounds / shape preconditions inside the
# kernels; python -m docagents_amd.ops.build --debug) instead of the -O3 library
_DEBUG = os.environ.get("DA_KERNELS_DEBUG", "0") == "1"
_LIB_PATH = Path(__file__).resolve().parent / ("_da_kernels_debug.so" if _DEBUG else "_da_kernels.so")

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_SWIGLU, EPI_RESID = 0, 1, 2, 3, 4
EPI_ROPE = 6  # gemm8p only: QKV + RoPE + KV-cache write

c_longlong = ctypes.c_longlong
c_void_p, c_int, c_float, c_uint, c_size_t = (ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                             ctypes.c_uint, ctypes.c_size_t)

_SIGS = {
    "da_gemm_bf16": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                     c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p],
    "da_gemm_rope": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int] + [c_void_p] * 5
                    + [c_int] * 5 + [c_void_p],
    "da_gemm_fp8": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                    c_int, c_int, c_int, c_int, c_void_p],
    "da_quant_fp8_rows": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "da_layernorm_q": [c_void_p] * 7 + [c_int, c_int, c_float, c_void_p],
    "da_bert_embed_ln_q": [c_void_p] * 11 + [c_int, c_int, c_float, c_void_p],
    "da_gemm_resid_rmsnorm": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_int, c_void_p],
    "da_rmsnorm": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p],
    "da_swiglu_interleaved": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p],
    "da_layernorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    "da_bert_embed_ln": [c_void_p] * 9 + [c_int, c_int, c_float, c_void_p],
    "da_embed": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "da_pool_l2norm": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "da_rope_cache": [c_void_p] * 6 + [c_int] * 6 + [c_void_p],
    "da_sample": [c_void_p, c_int, c_int, c_int, c_float, c_uint, c_uint] + [c_void_p] * 9
                 + [c_int] * 5 + [c_void_p],
    "da_flash_attn_v2": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int,
                         c_int, c_int, c_int, c_int, c_float, c_void_p, c_int, c_void_p, c_void_p, c_longlong,
                         c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "da_malloc_uncached": [c_longlong, ctypes.POINTER(c_void_p)],
    "da_gemm_dk": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                   c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p],
    "da_gemm_dk_parts": [c_int],
    "da_gemm_dk_splitk": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                          c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_void_p],
    "da_decode_attn": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                       c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                       c_int, c_void_p],
    "da_topk_dense": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_float, c_int,
                      c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "da_topk_dense_stream": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_float, c_int,
                             c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "da_topk_ranges": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                       c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "da_topk_merge": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "da_kmeans_accum": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "da_sample_partial": [c_void_p, c_int, c_int, c_int, c_int, c_float, c_uint, c_uint, c_void_p, c_void_p, c_void_p],
    "da_sample_chunked": [c_void_p, c_int, c_int, c_int, c_float, c_uint, c_uint] + [c_void_p] * 10
                         + [c_int] * 5 + [c_void_p],
    "da_sample_finalize": [c_void_p, c_int, c_int] + [c_void_p] * 8 + [c_int] * 5 + [c_void_p],
    "da_stream_create_cumask": [c_uint, ctypes.POINTER(c_uint), ctypes.POINTER(c_void_p)],
    "da_stream_get_cumask": [c_void_p, c_uint, ctypes.POINTER(c_uint)],
    "da_stream_destroy": [c_void_p],
    "da_device_cu_count": [c_int, ctypes.POINTER(c_int)],
    "da_placement_probe": [c_void_p, c_int, c_longlong, c_void_p],
    "da_spin": [c_int, c_void_p, c_void_p],
    "da_gemm8p_persist": [c_int],
    "da_gemm4w_variant": [c_int],
    "da_gemm_f16": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                    c_void_p],
    "da_flash_attn_f16": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                          c_int, c_int, c_float, c_void_p, c_int, c_void_p],
    "da_layernorm_f16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    "da_bert_embed_ln_f16": [c_void_p] * 9 + [c_int, c_int, c_float, c_void_p],
    "da_pool_l2norm_f16": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
}


class KernelLibraryMissing(RuntimeError):
    pass


class KernelError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load (building on first use if sources are newer) the kernel library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if os.environ.get("DA_BUILD_ON_IMPORT", "1") == "1":
            try:
                from .build import build
                build(debug=_DEBUG)
            except Exception as e:  # noqa: BLE001 - fall through to the explicit check below
                if not _LIB_PATH.exists():
                    raise KernelLibraryMissing(f"cannot build {_LIB_PATH}: {e}") from e
        if not _LIB_PATH.exists():
            raise KernelLibraryMissing(f"{_LIB_PATH} not built; run python -m docagents_amd.ops.build")
        import torch.cuda  # noqa: F401 - make sure torch's HIP runtime is loaded first
        L = ctypes.CDLL(str(_LIB_PATH))
        for name, argt in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = c_int
        L.da_topk_dense_ws.argtypes = [c_int, c_int, c_int, c_int]
        L.da_topk_dense_ws.restype = c_size_t
        L.da_topk_stream_ws.argtypes = [c_int, c_int, c_int, c_int]
        L.da_topk_stream_ws.restype = c_size_t
        _LIB = L
        return L


def available() -> bool:
    return torch.cuda.is_available() and _LIB_PATH.exists()


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc: int, name: str):
    if rc != 0:
        raise KernelError(f"{name} failed with hipError {rc}")


def _req(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


def _bf16_cuda(t, name):
    _req(t.is_cuda, f"{name} must be on GPU")
    _req(t.dtype == torch.bfloat16, f"{name} must be bf16, got {t.dtype}")


def _i32(t, name):
    _req(t.is_cuda and t.dtype == torch.int32 and t.is_contiguous(), f"{name} must be contiguous int32 on GPU")


# ----------------------------------------------------------------------------------- GEMM
_WS = {}
_ROLE = threading.local()


@contextlib.contextmanager
def workspace_role(name: str):
    """Kernels launched inside this context use the split-K / decode workspace of ``name``
    instead of the default one. Two phases that run CONCURRENTLY on different streams (the
    serving pipeline's prefill lane next to a replaying decode graph) must not share scratch:
    the decode graph captured the default workspace's pointer."""
    prev = getattr(_ROLE, "name", "main")
    _ROLE.name = name
    try:
        yield
    finally:
        _ROLE.name = prev


def workspace_buffer(device):
    """The current role's workspace tensor on ``device`` (None before its first use): callers that
    capture graphs check it is the same object after their captures (a grown workspace frees the
    buffer earlier captures point at)."""
    device = torch.device(device)
    key = (device.index if device.index is not None else torch.cuda.current_device(), getattr(_ROLE, "name", "main"))
    return _WS.get(key)


def _workspace(nbytes: int, device) -> torch.Tensor:
    key = (device.index if device.index is not None else torch.cuda.current_device(), getattr(_ROLE, "name", "main"))
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def gemv_fusable(M: int, N: int, K: int, epi: int = EPI_NONE) -> bool:
    """True when gemm() runs the batch-1 GEMV (which can also fuse the input RMSNorm)."""
    return M == 1 and K % 512 == 0 and N % 4 == 0 and (epi != EPI_SWIGLU or N % 32 == 0)


def gemm(a: torch.Tensor, w: torch.Tensor, bias=None, epi: int = EPI_NONE, resid=None, out=None,
         tile: int = 0, splits: int = 0, rms=None) -> torch.Tensor:
    """out[M, N'] = epi(a[M, K] @ w[N, K]^T). N' = N/2 for EPI_SWIGLU (w rows interleaved by 16).
    rms = (gamma, eps): ``a`` is the raw residual stream and RMSNorm(a) * gamma is fused into the
    GEMV (M == 1 only, see gemv_fusable); gamma None = unit gain (folded into ``w``)."""
    _bf16_cuda(a, "a"); _bf16_cuda(w, "w")
    _req(a.dim() == 2 and w.dim() == 2, "gemm expects 2-D operands")
    M, K = a.shape
    N, K2 = w.shape
    _req(K == K2, f"K mismatch {K} vs {K2}")
    _req(K % 64 == 0, f"K={K} must be a multiple of 64")
    _req(N % 8 == 0, f"N={N} must be a multiple of 8")
    _req(a.stride(1) == 1 and a.stride(0) % 8 == 0 and a.stride(0) >= K, "a must be row-major, 16-B aligned rows")
    _req(w.is_contiguous(), "w must be contiguous")
    _req(a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0, "operands must be 16-B aligned")
    nout = N // 2 if epi == EPI_SWIGLU else N
    if epi == EPI_SWIGLU:
        _req(N % 32 == 0, "SwiGLU needs N % 32 == 0")
    if out is None:
        out = torch.empty((M, nout), dtype=torch.bfloat16, device=a.device)
    _bf16_cuda(out, "out")
    _req(out.shape == (M, nout) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "bad out")
    if bias is not None:
        _bf16_cuda(bias, "bias"); _req(bias.numel() == N and bias.is_contiguous(), "bias must be [N]")
        _req(epi in (EPI_BIAS, EPI_GELU, EPI_RESID), "bias only with BIAS/GELU/RESID epilogues")
    ldr = 0
    if epi == EPI_RESID:
        _req(resid is not None, "EPI_RESID needs resid")
        _bf16_cuda(resid, "resid")
        _req(resid.shape == (M, N) and resid.stride(1) == 1 and resid.stride(0) % 8 == 0, "bad resid")
        ldr = resid.stride(0)
    if M == 0:
        return out
    if (tile == 12 or (tile == 0 and splits <= 0)) and rms is None and dk_fusable(M, N, K, epi):
        return gemm_dk(a, w, epi=epi, bias=bias, resid=resid, out=out)
    if tile == 0 and splits <= 0 and gemv_fusable(M, N, K, epi):
        tile, splits = 6, 1  # batch-1 decode: weight-streaming GEMV, one launch, no split-K workspace
    gamma, eps = (None, 0.0) if rms is None else rms  # rms = (gain or None for unit gain, eps > 0)
    if rms is not None:
        _req(tile == 6, "fused RMSNorm needs the M == 1 GEMV path")
        _req(eps > 0, "fused RMSNorm needs eps > 0")
        if gamma is not None:
            _bf16_cuda(gamma, "gamma"); _req(gamma.numel() == K, "gamma must be [K]")
    if splits <= 0:
        if tile == 0 and M < 640:
            tile = _decode_tile(M, N)
        splits = _auto_splits(M, N, K) if tile in (0, 2, 3) or (tile == 9 and M <= 128) else 1
    ws = None
    if splits > 1:
        ws = _workspace(splits * M * N * 4, a.device)
    rc = lib().da_gemm_bf16(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), _ptr(bias), _ptr(resid), ldr,
                            M, N, K, epi, tile, splits, _ptr(ws), _ptr(gamma), float(eps), _stream())
    _check(rc, "gemm")
    return out


# Decode GEMMs with 2..64 rows: gemm_dk (csrc/gemm_dk.hip: K split across the 4 waves of a
# workgroup and summed through LDS, no split-K partials, no reduce launch). False: the 64x128 /
# 32x128 tiles + split-K + reduce (bench/ab_arms.py DA_DECODE_DK=0).
DECODE_DK = True
# 33..64 rows keep the gemm_dk layer structure (norms deferred into the consumer) on the split-K
# tiles: the narrow dk tiles re-read the activation block once per 16-64 weight rows there
# (bench/midm_chain.py, profiles/r3/dk/), so gemm_dk() routes those rows to da_gemm_dk_splitk
# (reduce + residual + row sums of squares; the consumer's reduce applies the row scale)
DK_MAX_M = 64
DK_SPLITK_ABOVE = 32


def dk_fusable(M: int, N: int, K: int, epi: int = EPI_NONE) -> bool:
    """True when gemm() runs a decode-sized product on gemm_dk (no split-K)."""
    return (DECODE_DK and 2 <= M <= DK_MAX_M and K % 256 == 0 and N % 16 == 0
            and epi in (EPI_NONE, EPI_BIAS, EPI_RESID, EPI_SWIGLU) and (epi != EPI_SWIGLU or N % 32 == 0))


def _dk_splitk(M: int, N: int) -> bool:
    return DK_SPLITK_ABOVE < M <= 64 and N % 512 == 0


def _dk_splits(N: int, K: int) -> int:
    """Split-K of the 33..64-row route (64x128 tiles): the largest of 2, 3, 4, 6, 8, 12, 16 that keeps
    the grid within one round of 256 workgroups and >= 4 K-steps of 64 per split; at least 2 (the
    reduce carries the epilogue). 3 is the point of this list: the Phi-3 QKV projection (72 tiles)
    18.7 us at 3 splits vs 21.8 at 2 and 25.7 at 4 (bench/splitk_m64.py, profiles/r3/splitk_m64.txt)."""
    tiles, ks = (N + 127) // 128, K // 64
    best = 2
    for s in (2, 3, 4, 6, 8, 12, 16):
        if ks % s == 0 and ks // s >= 4 and tiles * s <= 256:
            best = s
    return best if ks % best == 0 else 2


def dk_parts(N: int, M: int = 0) -> int:
    """Row-norm partial sums an EPI_RESID gemm_dk of width N and M rows writes (the consumer's part
    count): one per dk output tile, or one per 512 columns on the 33..64-row split-K route."""
    if _dk_splitk(M, N):
        return N // 512
    return int(lib().da_gemm_dk_parts(N))


def gemm_dk(a, w, epi: int = EPI_NONE, bias=None, resid=None, out=None, norm_in=None, ssq_out=None):
    """Decode-sized product (1 <= M <= 64) in one launch without split-K:
    out = epi(rownorm(a) @ w^T). norm_in = (ssq, parts, eps): ``a`` is the raw residual stream and
    each row is scaled by rsqrt(sum of ssq[:parts, row] / K + eps) first (bf16-rounded, as the
    rmsnorm kernel would; RMSNorm gains folded into w). ssq_out (EPI_RESID only): fp32
    [dk_parts(N), 64] receives the per-part sums of squares of the new rows, for the next consumer."""
    _bf16_cuda(a, "a"); _bf16_cuda(w, "w")
    M, K = a.shape
    N = w.shape[0]
    _req(1 <= M <= 64 and K % 256 == 0 and N % 16 == 0 and w.shape[1] == K, f"gemm_dk shape M={M} N={N} K={K}")
    _req(a.stride(1) == 1 and a.stride(0) % 8 == 0 and w.is_contiguous(), "gemm_dk layout")
    _req(a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0, "operands must be 16-B aligned")
    nout = N // 2 if epi == EPI_SWIGLU else N
    if out is None:
        out = torch.empty((M, nout), dtype=torch.bfloat16, device=a.device)
    _req(out.shape == (M, nout) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "bad out")
    ldr = 0
    if epi == EPI_RESID:
        _req(resid is not None and resid.shape == (M, N) and resid.stride(1) == 1 and resid.stride(0) % 8 == 0,
             "bad resid")
        ldr = resid.stride(0)
    ssq, parts, eps = (None, 0, 0.0) if norm_in is None else norm_in
    if ssq is not None:
        _req(ssq.dtype == torch.float32 and ssq.is_contiguous() and ssq.numel() >= parts * 64, "bad ssq_in")
    if ssq_out is not None:
        _req(epi == EPI_RESID and ssq_out.dtype == torch.float32 and ssq_out.is_contiguous()
             and ssq_out.numel() >= dk_parts(N, M) * 64, "bad ssq_out")
    if _dk_splitk(M, N) or (DK_SPLITK_ABOVE < M <= 64 and ssq_out is None):
        splits = _dk_splits(N, K)
        ws = _workspace(splits * M * N * 4, a.device)
        _check(lib().da_gemm_dk_splitk(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), _ptr(bias), _ptr(resid),
                                       ldr, M, N, K, epi, _ptr(ssq), parts, K, float(eps), _ptr(ssq_out), _ptr(ws),
                                       splits, _stream()), "gemm_dk_splitk")
        return out
    _check(lib().da_gemm_dk(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), _ptr(bias), _ptr(resid), ldr,
                            M, N, K, epi, _ptr(ssq), parts, K, float(eps), _ptr(ssq_out), _stream()), "gemm_dk")
    return out


# Every GEMM runs on the in-tree kernels: gemm8p (phase-split BMx256, csrc/gemm8p.hip) from 256
# rows, the 64x128 / 32x128 weight-streaming tiles + split-K below, the GEMV at batch 1. The
# vendor-library arms used for comparisons live in bench/ab_arms.py (same-box measurements:
# profiles/r2/ab_gemm8p_vs_hipblaslt.txt).


def gemm_rope(a, w, pos, cos_sin, H: int, Hkv: int, D: int, slot, k_cache, v_cache, out=None,
              kv_out: bool = True) -> torch.Tensor:
    """Prefill QKV projection: qkv = a @ w^T with RoPE applied to the q / k heads and the token's
    k / v written to the KV cache (cache [slots, Hkv, max_seq, D]) — one kernel (gemm8p EPI_ROPE)
    from 256 rows; shorter prefills run gemm + rope_cache (identical roundings). kv_out=False: the
    k / v columns of the result may be left unwritten (the attention reads the cache; see
    flash_attn_varlen kv_cache) — only the q columns are defined."""
    _bf16_cuda(a, "a"); _bf16_cuda(w, "w"); _i32(pos, "pos"); _i32(slot, "slot")
    M, K = a.shape
    N = w.shape[0]
    _req(N == (H + 2 * Hkv) * D and w.shape[1] == K and D % 8 == 0, "qkv weight shape")
    _req(pos.numel() >= M and slot.numel() >= M, "pos / slot length")
    _req(cos_sin.dtype == torch.float32 and cos_sin.is_contiguous() and cos_sin.shape[1] == D // 2, "cos_sin")
    _req(k_cache.is_contiguous() and v_cache.is_contiguous() and k_cache.shape == v_cache.shape
         and k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[3] == D, "caches")
    if M < 256 or K % 64 or K < 128 or a.stride(1) != 1 or a.stride(0) % 8 or not w.is_contiguous():
        qkv = gemm(a, w, out=out)
        return rope_cache(qkv, pos, cos_sin, H, Hkv, D, slot=slot, k_cache=k_cache, v_cache=v_cache)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    _req(out.shape == (M, N) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "bad out")
    _check(lib().da_gemm_rope(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), M, N, K, _ptr(pos), _ptr(slot),
                              _ptr(cos_sin), _ptr(k_cache), _ptr(v_cache), H, Hkv, D, k_cache.shape[2], int(kv_out),
                              _stream()),
           "gemm_rope")
    return out


FP8 = torch.float8_e4m3fn  # OCP e4m3 (gfx950), not the MI300 fnuz variant


def quant_fp8(x: torch.Tensor, out=None, scale=None):
    """Per-row dynamic e4m3 quantisation: returns (q [M, K] float8_e4m3fn, scale [M] fp32)."""
    _bf16_cuda(x, "x")
    _req(x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.shape[1] % 8 == 0, "x layout")
    M, K = x.shape
    if out is None:
        out = torch.empty((M, K), dtype=FP8, device=x.device)
    if scale is None:
        scale = torch.empty(M, dtype=torch.float32, device=x.device)
    _req(out.dtype == FP8 and out.shape == (M, K) and out.stride(1) == 1 and out.stride(0) % 16 == 0, "bad out")
    _req(scale.dtype == torch.float32 and scale.numel() >= M, "bad scale")
    _check(lib().da_quant_fp8_rows(_ptr(x), x.stride(0), M, K, _ptr(out), out.stride(0), _ptr(scale), _stream()),
           "quant_fp8")
    return out, scale


def quant_weight_fp8(w: torch.Tensor):
    """Per-output-channel e4m3 weight quantisation (host-side torch; done once at load)."""
    wf = w.float()
    sw = (wf.abs().amax(dim=1) / 448.0).clamp_min(1e-30)
    return (wf / sw[:, None]).clamp(-448, 448).to(FP8).contiguous(), sw.contiguous()


def gemm_fp8(aq, sa, wq, sw, bias=None, epi: int = EPI_NONE, resid=None, out=None) -> torch.Tensor:
    """out[M, N] = epi((aq . wq^T) * sa[:, None] * sw[None, :]) with e4m3 operands (256x256 MFMA tile)."""
    _req(aq.is_cuda and aq.dtype == FP8 and wq.dtype == FP8, "fp8 operands expected")
    M, K = aq.shape
    N, K2 = wq.shape
    _req(K == K2 and K % 128 == 0 and N % 8 == 0, f"fp8 gemm shape M={M} N={N} K={K}")
    _req(aq.stride(1) == 1 and aq.stride(0) % 16 == 0 and wq.is_contiguous(), "fp8 operand layout")
    _req(aq.data_ptr() % 16 == 0 and wq.data_ptr() % 16 == 0, "operands must be 16-B aligned")
    _req(sa.dtype == torch.float32 and sa.numel() >= M and sw.dtype == torch.float32 and sw.numel() == N, "scales")
    nout = N // 2 if epi == EPI_SWIGLU else N
    if out is None:
        out = torch.empty((M, nout), dtype=torch.bfloat16, device=aq.device)
    _bf16_cuda(out, "out")
    _req(out.shape == (M, nout) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "bad out")
    if bias is not None:
        _bf16_cuda(bias, "bias"); _req(bias.numel() == N, "bias must be [N]")
    ldr = 0
    if epi == EPI_RESID:
        _req(resid is not None and resid.shape == (M, N) and resid.stride(1) == 1, "bad resid")
        ldr = resid.stride(0)
    if M == 0:
        return out
    _check(lib().da_gemm_fp8(_ptr(aq), aq.stride(0), _ptr(wq), _ptr(sa), _ptr(sw), _ptr(out), out.stride(0),
                             _ptr(bias), _ptr(resid), ldr, M, N, K, epi, _stream()), "gemm_fp8")
    return out


def gemm_resid_norm(a, w, resid, gamma, eps: float, out=None, h_out=None, bias=None, tile: int = 0, splits: int = 0):
    """Decode layer tail (M <= 128): out = resid + a @ w^T (+ bias) — the new residual stream — and
    h_out = RMSNorm(out) * gamma, with the norm fused into the split-K reduction. Returns h_out."""
    _bf16_cuda(a, "a"); _bf16_cuda(w, "w"); _bf16_cuda(resid, "resid"); _bf16_cuda(gamma, "gamma")
    M, K = a.shape
    N = w.shape[0]
    _req(M <= 128 and K % 64 == 0 and N % 8 == 0 and N <= 8192 and w.shape[1] == K, "gemm_resid_norm shape")
    _req(a.stride(1) == 1 and a.stride(0) % 8 == 0 and w.is_contiguous() and gamma.numel() == N, "layout")
    _req(resid.shape == (M, N) and resid.stride(1) == 1, "bad resid")
    out = resid if out is None else out
    if h_out is None:
        h_out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if M == 0:
        return h_out
    tile = tile or (9 if M > 64 else _decode_tile(M))  # the fused reduce + norm: 128x64 tile above 64 rows
    if splits <= 0:
        splits = _auto_splits(M, N, K)
    ws = _workspace(splits * M * N * 4, a.device)
    _check(lib().da_gemm_resid_rmsnorm(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), _ptr(bias),
                                       _ptr(resid), resid.stride(0), M, N, K, tile, splits, _ptr(ws), _ptr(gamma),
                                       float(eps), _ptr(h_out), h_out.stride(0), _stream()), "gemm_resid_norm")
    return h_out


def _decode_tile(M: int, N: int = 0) -> int:
    """Decode-sized M: 32x128 tiles up to 32 rows, 64x128 to 64; 65..128 rows (a batch-128 decode
    step): N >= 8192 (QKV, gate/up, LM head: >= 128 weight tiles) the 64x128 tile over the two row
    blocks without split-K, else one 128x64 weight-streaming tile per 64 weight rows with split-K
    (profiles/r5/midm/decode_gemm_sweep_m128.txt, weights cold: QKV 28.0 vs 33.5 us, gate/up 30.5 vs
    47.4 us at 128 rows vs the 128x64 tile at split 4; O / down best on the 128x64 tile at split 4);
    129..639 rows the 64x128 tile over ceil(M/64) row blocks."""
    if M <= 32:
        return 3
    if 64 < M <= 128:
        return 2 if N >= 8192 else 9
    return 2


def _auto_splits(M: int, N: int, K: int) -> int:
    """Split-K for decode-sized M: the largest power of two keeping <= 256 workgroups (one per CU)
    and >= 4 K-steps per split. With 4 k-tiles in flight per workgroup (gemm.hip PF) a tile needs
    fewer splits to cover HBM latency, and fewer splits = fewer partial bytes to reduce. From a
    graph-replayed sweep with weights streamed cold from HBM, as in a real decode step
    (profiles/decode_gemm_prefetch_sweep_r1.jsonl: matches the best split on 17 of 20 Phi-3 /
    Llama-3-8B shapes at M = 16 / 64, within 0.7 us on the rest)."""
    if M >= 640:
        return 1
    ksteps = K // 64
    if 64 < M <= 128:  # (see _decode_tile) wide N: no split; else 4 splits, fewer if K is short
        if N >= 8192:
            return 1
        s = 4
        while s > 1 and (ksteps % s or ksteps // s < 4):
            s //= 2
        return s
    tiles = math.ceil(M / (32 if _decode_tile(M) == 3 else 64)) * math.ceil(N / 128)
    # 65..639 rows run the 64x128 tile over ceil(M/64) row blocks (the row blocks of one weight tile
    # share it through L2): up to 4 workgroups per CU below 256 rows, 2.5 from 256 (32-layer Phi-3
    # chain, bench/midm_chain.py, profiles/r2/midm_chain.txt: split 4 best at M = 65 / 128, 2 at 192 /
    # 256, 1 from 384)
    cap = 256 if M <= 64 else (1024 if M < 256 else 640)
    s = 1
    while tiles * s * 2 <= cap and ksteps % (s * 2) == 0 and ksteps // (s * 2) >= 4:
        s *= 2
    return s


# ------------------------------------------------------------------------------ norms etc.
def rmsnorm(x, w, eps: float, resid=None, out=None):
    _bf16_cuda(x, "x"); _bf16_cuda(w, "w")
    M, D = x.shape
    _req(x.stride(1) == 1 and x.stride(0) % 8 == 0 and D % 8 == 0, "x must be row-major, D % 8 == 0")
    _req(w.numel() == D, "w must be [D]")
    if resid is not None:
        _bf16_cuda(resid, "resid"); _req(resid.is_contiguous() and resid.shape == (M, D), "resid must be [M, D]")
    if out is None:
        out = torch.empty((M, D), dtype=torch.bfloat16, device=x.device)
    _req(out.stride(1) == 1 and out.stride(0) % 8 == 0, "bad out")
    _check(lib().da_rmsnorm(_ptr(x), x.stride(0), _ptr(resid), _ptr(w), _ptr(out), out.stride(0), M, D,
                            float(eps), _stream()), "rmsnorm")
    return out


def layernorm(x, g, b, eps: float, resid=None, out=None, fp8_out: bool = False):
    """LayerNorm; with ``fp8_out`` also returns the row-quantised e4m3 copy and its scales
    (fused: the row is quantised from registers) -> (y, yq, yscale)."""
    _bf16_cuda(x, "x")
    M, D = x.shape
    _req(x.is_contiguous() and D % 8 == 0, "x must be contiguous, D % 8 == 0")
    if resid is not None:
        _req(resid.is_contiguous() and resid.shape == x.shape, "bad resid")
    if out is None:
        out = torch.empty_like(x)
    if fp8_out:
        yq = torch.empty((M, D), dtype=FP8, device=x.device)
        ys = torch.empty(M, dtype=torch.float32, device=x.device)
        _check(lib().da_layernorm_q(_ptr(x), _ptr(resid), _ptr(g), _ptr(b), _ptr(out), _ptr(yq), _ptr(ys), M, D,
                                    float(eps), _stream()), "layernorm_q")
        return out, yq, ys
    _check(lib().da_layernorm(_ptr(x), _ptr(resid), _ptr(g), _ptr(b), _ptr(out), M, D, float(eps), _stream()),
           "layernorm")
    return out


def bert_embed_ln(ids, positions, types, word, pos, type_, g, b, eps: float, out=None, fp8_out: bool = False):
    _i32(ids, "ids"); _i32(positions, "positions")
    if types is not None:
        _i32(types, "types")
    T = ids.numel()
    D = word.shape[1]
    _req(positions.numel() == T, "positions length")
    if out is None:
        out = torch.empty((T, D), dtype=torch.bfloat16, device=ids.device)
    if fp8_out:
        yq = torch.empty((T, D), dtype=FP8, device=ids.device)
        ys = torch.empty(T, dtype=torch.float32, device=ids.device)
        _check(lib().da_bert_embed_ln_q(_ptr(ids), _ptr(positions), _ptr(types), _ptr(word), _ptr(pos), _ptr(type_),
                                        _ptr(g), _ptr(b), _ptr(out), _ptr(yq), _ptr(ys), T, D, float(eps), _stream()),
               "bert_embed_ln_q")
        return out, yq, ys
    _check(lib().da_bert_embed_ln(_ptr(ids), _ptr(positions), _ptr(types), _ptr(word), _ptr(pos), _ptr(type_),
                                  _ptr(g), _ptr(b), _ptr(out), T, D, float(eps), _stream()), "bert_embed_ln")
    return out


def embed(ids, table, out=None):
    _i32(ids, "ids"); _bf16_cuda(table, "table")
    T, D = ids.numel(), table.shape[1]
    if out is None:
        out = torch.empty((T, D), dtype=torch.bfloat16, device=ids.device)
    _check(lib().da_embed(_ptr(ids), _ptr(table), _ptr(out), T, D, _stream()), "embed")
    return out


def pool_l2norm(h, cu_seqlens, mode: int = 0, out32=None, out16=None):
    _bf16_cuda(h, "h"); _i32(cu_seqlens, "cu_seqlens")
    B = cu_seqlens.numel() - 1
    D = h.shape[1]
    _req(h.is_contiguous(), "h contiguous")
    if out32 is None and out16 is None:
        out32 = torch.empty((B, D), dtype=torch.float32, device=h.device)
    _check(lib().da_pool_l2norm(_ptr(h), _ptr(cu_seqlens), B, D, mode, _ptr(out32), _ptr(out16), _stream()),
           "pool_l2norm")
    return out32 if out32 is not None else out16


def rope_cache(qkv, pos, cos_sin, H, Hkv, D, slot=None, k_cache=None, v_cache=None, rotate_q=True):
    """In-place RoPE on q and k heads of qkv [T, (H+2Hkv)*D]; optionally writes k/v into the cache."""
    _bf16_cuda(qkv, "qkv"); _i32(pos, "pos")
    T = qkv.shape[0]
    _req(qkv.is_contiguous() and qkv.shape[1] == (H + 2 * Hkv) * D, "qkv shape")
    _req(cos_sin.dtype == torch.float32 and cos_sin.is_contiguous() and cos_sin.shape[-1] == 2
         and cos_sin.shape[1] == D // 2, "cos_sin must be fp32 [max_pos, D/2, 2]")
    max_seq = 0
    if k_cache is not None:
        _i32(slot, "slot")
        _req(k_cache.is_contiguous() and v_cache.is_contiguous() and k_cache.shape == v_cache.shape, "caches")
        _req(k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[3] == D, "cache [S, Hkv, max_seq, D]")
        max_seq = k_cache.shape[2]
    _check(lib().da_rope_cache(_ptr(qkv), _ptr(pos), _ptr(slot), _ptr(cos_sin), _ptr(k_cache), _ptr(v_cache),
                               T, H, Hkv, D, max_seq, 1 if rotate_q else 0, _stream()), "rope_cache")
    return qkv


def flash_kv_cache_ok(D: int, causal: bool) -> bool:
    """True when flash_attn_varlen can read the sequences' own keys from the KV cache (kv_cache=)."""
    return causal and D == 96


def flash_attn_varlen(q, k, v, cu_seqlens, max_seqlen: int, H: int, Hkv: int, D: int, causal: bool,
                      scale: float | None = None, out=None, prefix=None, kv_cache=None):
    """q/k/v: 2-D [T, *] views with head h at columns h*D (strided views into a packed qkv are fine).
    prefix = (k_pre, v_pre, P): shared-prefix keys of every sequence, one KV-cache slot's
    [Hkv, max_seq, D] K and V (RoPE applied); query i of a sequence is key P + i.
    kv_cache = (k_cache, v_cache, slot, pos) (flash_kv_cache_ok only): the own keys of the sequence
    starting at token t are k_cache[slot[t], :, pos[t] + j] (slot / pos int32 per token, as the QKV
    projection wrote them); k / v are then ignored (None allowed)."""
    kc = vc = ks = kpos = None
    if kv_cache is not None:
        kc, vc, ks, kpos = kv_cache
        _req(flash_kv_cache_ok(D, causal), "kv_cache: causal D = 96 only")
        _bf16_cuda(kc, "k_cache"); _bf16_cuda(vc, "v_cache"); _i32(ks, "slot"); _i32(kpos, "pos")
        _req(kc.is_contiguous() and vc.is_contiguous() and kc.shape == vc.shape and kc.dim() == 4
             and kc.shape[1] == Hkv and kc.shape[3] == D, "caches [slots, Hkv, max_seq, D]")
        _req(ks.numel() >= q.shape[0] and kpos.numel() >= q.shape[0], "slot / pos per token")
        k = v = q  # unused by the kernel in this mode
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _bf16_cuda(t, n)
        _req(t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0, f"{n} layout")
    _i32(cu_seqlens, "cu_seqlens")
    _req(D in (32, 64, 96, 128), f"head dim {D} unsupported")
    _req(H % Hkv == 0, "H % Hkv")
    T = q.shape[0]
    if out is None:
        out = torch.empty((T, H * D), dtype=torch.bfloat16, device=q.device)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    B = cu_seqlens.numel() - 1
    kp = vp = None
    hstride, P = 0, 0
    if prefix is not None:
        kp, vp, P = prefix
        P = int(P)
        _bf16_cuda(kp, "k_pre"); _bf16_cuda(vp, "v_pre")
        _req(kp.dim() == 3 and kp.shape == vp.shape and kp.shape[0] == Hkv and kp.shape[2] == D
             and kp.is_contiguous() and vp.is_contiguous() and 0 <= P <= kp.shape[1], "prefix K/V [Hkv, max_seq, D]")
        hstride = kp.shape[1] * D
    if kc is not None:
        _req(prefix is None or kp.shape[1] == kc.shape[2], "prefix and caches differ in max_seq")
        hstride = kc.shape[2] * D
    _check(lib().da_flash_attn_v2(_ptr(q), _ptr(k), _ptr(v), q.stride(0), k.stride(0), v.stride(0),
                                  _ptr(cu_seqlens), B, int(max_seqlen), H, Hkv, D, int(causal), float(scale),
                                  _ptr(out), out.stride(0), _ptr(kp), _ptr(vp), hstride, P, _ptr(ks), _ptr(kpos),
                                  _ptr(kc), _ptr(vc), _stream()),
           "flash_attn_varlen")
    return out


# Split-KV partials merged inside the decode kernel by the last split of each (row, kv head)
# (False: separate combine launch; tests cover both). The ticket counters stay zero between
# launches; buffers are only ever added, never freed, so a captured graph's pointer stays valid.
_FUSED_COMBINE = True
_UC: dict = {}


class _RawBuf:
    """A device allocation outside PyTorch's allocator (uncached memory), as a ``_ptr``-able object."""

    def __init__(self, ptr: int, nbytes: int):
        self.ptr, self.nbytes = ptr, nbytes

    def data_ptr(self) -> int:
        return self.ptr


def _uncached(tag: str, nbytes: int, device) -> _RawBuf:
    """Zeroed uncached (L2-bypassing) device memory for cross-workgroup hand-offs (decode split
    partials + tickets). Grows by adding buffers, never frees: captured graphs keep their pointers."""
    key = (tag, device.index if device.index is not None else torch.cuda.current_device(),
           getattr(_ROLE, "name", "main"))
    bufs = _UC.setdefault(key, [])
    if not bufs or bufs[-1].nbytes < nbytes:
        n = max(nbytes, 1 << 20)
        p = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(lib().da_malloc_uncached(n, ctypes.byref(p)), "hipExtMallocWithFlags(uncached)")
        bufs.append(_RawBuf(p.value, n))
    return bufs[-1]


def _decode_split(B: int, Hkv: int, max_len: int, chunk: int):
    """(chunk, nsplit) of a decode-attention launch (static for a captured graph: from max_len)."""
    if chunk <= 0:
        # measured on MI355X (profiles/decode_attn_chunks_r1.txt): per-workgroup overhead dominates
        # small chunks; aim for ~768 workgroups, 512..4096 keys each
        want = max_len * B * Hkv / 768
        chunk = 512
        while chunk < want and chunk < 4096:
            chunk *= 2
    return chunk, max(1, math.ceil(max_len / chunk))


# Same-XCD split exchange of the batch-1..small-batch MHA decode attention (attention.hip, VAR bit 3):
# all splits of a (row, kv head) pair on one XCD, their partials and ticket in cached memory (L2
# round trips instead of uncached ones). It relies on the launch's workgroup -> XCD round-robin, so
# it is used only after the placement probe confirmed that on this device, and never once a
# CU-masked stream exists in the process (a masked queue need not dispatch round-robin over XCDs;
# ops/streams.py sets MASKED_STREAMS). DA_DECODE_XC=0 turns it off.
DECODE_XC = os.environ.get("DA_DECODE_XC", "1") != "0"
MASKED_STREAMS = False
_XC_PROBE: dict = {}


def decode_xc_ok(device) -> bool:
    """True when every workgroup w of a launch runs on XCD w % 8 here (placement probe, once per
    device; not during a graph capture, where the answer stays unknown = False)."""
    if not DECODE_XC or MASKED_STREAMS:
        return False
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _XC_PROBE:
        return _XC_PROBE[idx]
    if torch.cuda.is_current_stream_capturing():
        return False
    n = 1024
    out = torch.zeros(n * 4, dtype=torch.int32, device=device)
    _check(lib().da_placement_probe(_ptr(out), n, 0, _stream()), "placement_probe")
    xcc = out.view(n, 4)[:, 0].cpu().numpy()
    ok = bool(len(set(xcc.tolist())) == 8 and all(len(set(xcc[r::8].tolist())) == 1 for r in range(8)))
    _XC_PROBE[idx] = ok
    return ok


_COUNTERS: dict = {}


def _cached_counters(tag: str, n: int, device) -> torch.Tensor:
    """Zeroed int32 counters in ordinary device memory that stay allocated (captured graphs keep the
    pointer; the kernels leave them zero)."""
    key = (tag, device.index if device.index is not None else torch.cuda.current_device(),
           getattr(_ROLE, "name", "main"))  # per workspace role, like the uncached ones: concurrent lanes
    bufs = _COUNTERS.setdefault(key, [])
    if not bufs or bufs[-1].numel() < n:
        bufs.append(torch.zeros(max(n, 1024), dtype=torch.int32, device=device))
    return bufs[-1]


def _decode_checks(q, k_cache, v_cache, lens, slot, H, Hkv, D, max_len, pre, rope):
    _bf16_cuda(q, "q"); _i32(lens, "lens"); _i32(slot, "slot")
    _req(D in (64, 96, 128), "head dim")
    _req((H // Hkv) in (1, 2, 4, 8) and H % Hkv == 0, "GQA group must be 1/2/4/8")
    B = q.shape[0]
    _req(k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[3] == D, "cache shape")
    _req(max_len <= k_cache.shape[2], "max_len > cache capacity")
    if pre is not None:
        _i32(pre, "pre"); _req(pre.shape == (B, 2) and pre.is_contiguous(), "pre must be int32 [B, 2]")
    cs = ps = None
    if rope is not None:
        cs, ps = rope
        _req(H == Hkv and D % 8 == 0, "fused RoPE decode: MHA only")
        _i32(ps, "pos")
        _req(cs.dtype == torch.float32 and cs.is_contiguous() and cs.shape[1] == D // 2 and cs.shape[2] == 2, "cos_sin")
        _req(q.stride(1) == 1 and q.shape[1] >= (H + 2 * Hkv) * D, "fused RoPE decode needs the qkv row")
        _req(k_cache.is_contiguous() and v_cache.is_contiguous(), "caches must be contiguous")
    return cs, ps


def decode_attn(q, k_cache, v_cache, lens, slot, H, Hkv, D, max_len: int, chunk: int = 0, scale=None, out=None,
                pre=None, rope=None):
    """q [B, >=H*D] (row stride any multiple of 8); lens/slot int32 [B]; max_len = max(lens) or the
    cache capacity (host int, fixes the split count so the launch is graph-capturable).
    chunk = keys per workgroup (0 = auto: enough workgroups to fill 256 CUs, 4 waves x 64-key tiles).
    pre: optional int32 [B, 2] device tensor (P, prefix slot), P % 64 == 0: keys [0, P) of row b
    are the batch's shared prompt head, stored once in the prefix slot (read through the cache).
    rope = (cos_sin fp32 [max_pos, D/2, 2], pos int32 [B]), MHA only: q is the raw qkv row
    [B, (H + 2 Hkv) D]; the kernel applies RoPE to q and the new token's k and writes that token's
    k / v into the cache at pos (== lens - 1) — the decode step's rope_cache launch folded in."""
    cs, ps = _decode_checks(q, k_cache, v_cache, lens, slot, H, Hkv, D, max_len, pre, rope)
    chunk, nsplit = _decode_split(q.shape[0], Hkv, max_len, chunk)
    B = q.shape[0]
    ws = _workspace(B * H * nsplit * (D + 2) * 4, q.device)
    if out is None:
        out = torch.empty((B, H * D), dtype=torch.bfloat16, device=q.device)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    cnt = None
    xc = 0
    if _FUSED_COMBINE and nsplit > 1:
        if H == Hkv and B * Hkv <= 32 and (B * Hkv) % 8 == 0 and decode_xc_ok(q.device):
            xc = 1  # same-XCD exchange: ws (the role workspace) and counters in cached memory
            cnt = _cached_counters("decode_cnt_xc", B * Hkv, q.device)
        else:
            cnt = _uncached("decode_cnt", B * Hkv * 4, q.device)
            ws = _uncached("decode_ws", B * H * nsplit * (D + 2) * 4, q.device)
    _check(lib().da_decode_attn(_ptr(q), q.stride(0), _ptr(k_cache), _ptr(v_cache), _ptr(lens), _ptr(slot), _ptr(pre), B, H,
                                Hkv, D, k_cache.shape[2], chunk, nsplit, float(scale), _ptr(ws), _ptr(out), out.stride(0),
                                _ptr(cnt), _ptr(cs), _ptr(ps), xc, _stream()), "decode_attn")
    return out


# rows up to which sample() cuts the vocabulary over many workgroups (0: always one per row); at
# batch 64 one workgroup per row leaves 192 CUs idle too
SAMPLE_CHUNKED_MAX_B = 64
_SAMPLE_WS: dict = {}


def _sample_ws(nfloats: int, device) -> torch.Tensor:
    """Per-(device, workspace role) fp32 scratch of the chunked sampler. Grows by adding buffers and
    never frees one: a captured decode graph keeps pointing at the buffer it was captured with."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), getattr(_ROLE, "name", "main"))
    bufs = _SAMPLE_WS.setdefault(key, [])
    if not bufs or bufs[-1].numel() < nfloats:
        bufs.append(torch.empty(max(nfloats, 16384), dtype=torch.float32, device=device))
    return bufs[-1]


def sample(logits, temperature: float, seed: int, step: int = 0, out_tok=None, out_lp=None, conf=None,
           active=None, ctr=None, pos=None, lens=None, hist=None, start=None, eos=()):
    """Fused temperature sampler (see rope_sample.hip). Returns (tokens, logprobs)."""
    _bf16_cuda(logits, "logits")
    B, V = logits.shape
    _req(logits.stride(1) == 1 and logits.stride(0) % 8 == 0, "logits layout")
    dev = logits.device
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=dev)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=dev)
    if conf is not None:
        _req(conf.dtype == torch.float32 and conf.shape == (B, 2), "conf must be fp32 [B, 2]")
    for t, n in ((active, "active"), (ctr, "ctr"), (pos, "pos"), (lens, "lens"), (start, "start")):
        if t is not None:
            _i32(t, n); _req(t.numel() >= B, f"{n} too short")
    hist_ld = 0
    if hist is not None:
        _i32(hist, "hist"); _req(hist.dim() == 2 and hist.shape[0] >= B, "hist [B, n]")
        _req(pos is not None and start is not None, "hist needs pos and start")
        hist_ld = hist.shape[1]
    e = list(eos)[:4] + [-1] * (4 - min(4, len(eos)))
    if B <= SAMPLE_CHUNKED_MAX_B and V >= 4096:
        # few rows: the row is split over ceil(V / 1024) workgroups + a finalize launch (same token;
        # the batch-1 sampler took ~21 us on one CU, rope_sample.hip sample_chunk_kernel)
        ws = _sample_ws(B * ((V + 1023) // 1024) * 8, dev)
        _check(lib().da_sample_chunked(_ptr(logits), B, V, logits.stride(0), float(temperature), seed & 0xffffffff,
                                       step & 0xffffffff, _ptr(ctr), _ptr(ws), _ptr(out_tok), _ptr(out_lp),
                                       _ptr(conf), _ptr(active), _ptr(pos), _ptr(lens), _ptr(hist), _ptr(start),
                                       hist_ld, e[0], e[1], e[2], e[3], _stream()), "sample_chunked")
        return out_tok, out_lp
    _check(lib().da_sample(_ptr(logits), B, V, logits.stride(0), float(temperature), seed & 0xffffffff,
                           step & 0xffffffff, _ptr(ctr), _ptr(out_tok), _ptr(out_lp), _ptr(conf), _ptr(active),
                           _ptr(pos), _ptr(lens), _ptr(hist), _ptr(start), hist_ld, e[0], e[1], e[2], e[3],
                           _stream()), "sample")
    return out_tok, out_lp


def sample_partial(logits, temperature: float, seed: int, v0: int, step: int = 0, ctr=None, out=None):
    """Vocab-parallel sampling, rank side: logits [B, Vl] of the vocabulary slice starting at global
    index v0 -> stats fp32 [B, 8] = (best Gumbel score, best global index as int bits, local max,
    local sum exp(x - max), logit of the best, 0, 0, 0). See rope_sample.hip."""
    _bf16_cuda(logits, "logits")
    B, V = logits.shape
    _req(logits.stride(1) == 1, "logits rows must be contiguous")
    if ctr is not None:
        _i32(ctr, "ctr"); _req(ctr.numel() >= B, "ctr too short")
    if out is None:
        out = torch.empty((B, 8), dtype=torch.float32, device=logits.device)
    _req(out.dtype == torch.float32 and out.shape == (B, 8) and out.is_contiguous(), "stats must be fp32 [B, 8]")
    _check(lib().da_sample_partial(_ptr(logits), B, V, logits.stride(0), int(v0), float(temperature),
                                   seed & 0xffffffff, step & 0xffffffff, _ptr(ctr), _ptr(out), _stream()),
           "sample_partial")
    return out


def sample_finalize(gathered, ranks: int, out_tok=None, out_lp=None, conf=None, active=None, pos=None, lens=None,
                    hist=None, start=None, eos=()):
    """Vocab-parallel sampling, merge side: gathered fp32 [B, ranks * 8] (every rank's stats, rank
    order) -> the token / logprob / bookkeeping of ``sample`` on the full row."""
    _req(gathered.is_cuda and gathered.dtype == torch.float32 and gathered.is_contiguous(), "gathered fp32")
    B = gathered.shape[0]
    _req(gathered.shape == (B, 8 * ranks), f"gathered must be [B, {8 * ranks}]")
    dev = gathered.device
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=dev)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=dev)
    if conf is not None:
        _req(conf.dtype == torch.float32 and conf.shape == (B, 2), "conf must be fp32 [B, 2]")
    for t, n in ((active, "active"), (pos, "pos"), (lens, "lens"), (start, "start")):
        if t is not None:
            _i32(t, n); _req(t.numel() >= B, f"{n} too short")
    hist_ld = 0
    if hist is not None:
        _i32(hist, "hist"); _req(hist.dim() == 2 and hist.shape[0] >= B, "hist [B, n]")
        _req(pos is not None and start is not None, "hist needs pos and start")
        hist_ld = hist.shape[1]
    e = list(eos)[:4] + [-1] * (4 - min(4, len(eos)))
    _check(lib().da_sample_finalize(_ptr(gathered), B, ranks, _ptr(out_tok), _ptr(out_lp), _ptr(conf), _ptr(active),
                                    _ptr(pos), _ptr(lens), _ptr(hist), _ptr(start), hist_ld, e[0], e[1], e[2], e[3],
                                    _stream()), "sample_finalize")
    return out_tok, out_lp


# --------------------------------------------------------------------------- vector search
def topk_dense(X, Qv, K: int, thr: float, slots=None, bitmap=None, rows_per_block: int | None = None):
    """Exact top-K of Qv @ X^T per query with threshold and optional doc-slot bitmap [Q, W] int32."""
    _bf16_cuda(X, "X"); _bf16_cuda(Qv, "Qv")
    N, d = X.shape
    Q = Qv.shape[0]
    _req(X.is_contiguous() and Qv.is_contiguous() and Qv.shape[1] == d, "X/Qv layout")
    _req(d % 32 == 0 and 1 <= K <= 32, "d % 32 and 1 <= K <= 32")
    W = 0
    if slots is not None:
        _i32(slots, "slots")
        _req(slots.numel() >= N, "slots length")
    if bitmap is not None:
        _req(slots is not None, "bitmap needs slots")
        _req(bitmap.dtype == torch.int32 and bitmap.is_contiguous() and bitmap.shape[0] == Q, "bitmap [Q, W] int32")
        W = bitmap.shape[1]
    if d in (384, 768, 1024) and rows_per_block is None and N > 0 and Q <= 256:
        # the streaming scan (search-sized batches over a big shard; k-means assignment, with the
        # rows as the queries, keeps the query-major tiles below): ~16 waves of rows per CU over
        # the chip (256 CUs), >= 64 rows each
        rpw = max(64, math.ceil(N / (256 * 16) / 16) * 16)
        ws = _workspace(int(lib().da_topk_stream_ws(N, Q, K, rpw)), X.device)
        out_s = torch.empty((Q, K), dtype=torch.float32, device=X.device)
        out_i = torch.empty((Q, K), dtype=torch.int32, device=X.device)
        _check(lib().da_topk_dense_stream(_ptr(X), N, d, _ptr(slots), _ptr(Qv), Q, _ptr(bitmap), W, float(thr), K,
                                          rpw, _ptr(ws), _ptr(out_s), _ptr(out_i), _stream()), "topk_dense_stream")
        return out_s, out_i
    if rows_per_block is None:
        qt = math.ceil(Q / 16)
        nblk = max(1, min(math.ceil(N / 256), max(1, 1024 // qt)))
        rows_per_block = max(64, math.ceil(math.ceil(N / nblk) / 64) * 64)
    nblk = max(1, math.ceil(N / rows_per_block))
    ws = _workspace(nblk * Q * K * 8, X.device)
    out_s = torch.empty((Q, K), dtype=torch.float32, device=X.device)
    out_i = torch.empty((Q, K), dtype=torch.int32, device=X.device)
    _check(lib().da_topk_dense(_ptr(X), N, d, _ptr(slots), _ptr(Qv), Q, _ptr(bitmap), W, float(thr), K,
                               rows_per_block, _ptr(ws), _ptr(out_s), _ptr(out_i), _stream()), "topk_dense")
    return out_s, out_i


def topk_ranges(X, Qv, ranges, range_off, K: int, thr: float, max_rows: int, slots=None, bitmap=None,
                rows_per_split: int = 512):
    """Top-K per query over its own row ranges. ranges int32 [R, 2], range_off int32 [Q+1];
    max_rows = max total rows of any query (host int) — sets the split count."""
    _bf16_cuda(X, "X"); _bf16_cuda(Qv, "Qv")
    N, d = X.shape
    Q = Qv.shape[0]
    _req(d % 8 == 0 and d <= 4096 and 1 <= K <= 32, "d / K limits")
    _i32(ranges, "ranges"); _i32(range_off, "range_off")
    _req(range_off.numel() == Q + 1, "range_off length")
    W = 0
    if slots is not None:
        _i32(slots, "slots")
        _req(slots.numel() >= N, "slots length")
    if bitmap is not None:
        _req(slots is not None, "bitmap needs slots")
        _req(bitmap.dtype == torch.int32 and bitmap.shape[0] == Q, "bitmap")
        W = bitmap.shape[1]
    splits = max(1, math.ceil(max_rows / rows_per_split))
    ws = _workspace(splits * Q * K * 8, X.device)
    out_s = torch.empty((Q, K), dtype=torch.float32, device=X.device)
    out_i = torch.empty((Q, K), dtype=torch.int32, device=X.device)
    _check(lib().da_topk_ranges(_ptr(X), d, _ptr(slots), _ptr(Qv), Q, _ptr(ranges), _ptr(range_off), _ptr(bitmap),
                                W, float(thr), K, splits, rows_per_split, _ptr(ws), _ptr(out_s), _ptr(out_i),
                                _stream()), "topk_ranges")
    return out_s, out_i


def topk_merge(cand_s, cand_i, K: int):
    """cand [P, Q, K] (consumed) -> [Q, K]."""
    _req(cand_s.dtype == torch.float32 and cand_i.dtype == torch.int32, "dtypes")
    P, Q, K2 = cand_s.shape
    _req(K2 == K, "K mismatch")
    cs, ci = cand_s.contiguous().clone(), cand_i.contiguous().clone()
    out_s = torch.empty((Q, K), dtype=torch.float32, device=cs.device)
    out_i = torch.empty((Q, K), dtype=torch.int32, device=cs.device)
    _check(lib().da_topk_merge(_ptr(cs), _ptr(ci), P, Q, K, _ptr(out_s), _ptr(out_i), _stream()), "topk_merge")
    return out_s, out_i


def kmeans_accum(X, assign, sums, counts):
    _bf16_cuda(X, "X"); _i32(assign, "assign")
    N, d = X.shape
    _req(sums.dtype == torch.float32 and sums.shape[1] == d and counts.dtype == torch.float32, "sums/counts fp32")
    _check(lib().da_kmeans_accum(_ptr(X), N, d, _ptr(assign), _ptr(sums), _ptr(counts), _stream()), "kmeans_accum")


def reserve_workspace(nbytes: int, device=None) -> None:
    """Pre-size the shared split-K / decode workspace. Must be called before capturing HIP graphs
    so the captured kernels keep pointing at a live buffer."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    _workspace(nbytes, dev)


def spin(us: int, device=None) -> None:
    """Hold the current stream busy for ``us`` microseconds (one wave polling the wall clock;
    bounded to 10 s). Test helper: work queued behind it on this stream is provably still pending."""
    _req(0 <= us <= 10_000_000, "spin: 0 <= us <= 1e7")
    _check(lib().da_spin(int(us), None, _stream()), "da_spin")


def gemm8p_persist(on: int = -1) -> int:
    """Persistent tile loop of the prefill GEMM (one workgroup per CU walking its XCD's tiles) on
    (1) / off (0) for later launches; -1 only queries. Returns the previous setting."""
    return int(lib().da_gemm8p_persist(int(on)))


def gemm4w_variant(v: int = -1) -> int:
    """Schedule of the four-wave 256x256 kernel (tile 13, csrc/gemm4w.hip) where K / 64 is even and
    >= 4: 0 = three fragment sets, two barriers per K-tile (default), 1 = two sets, 2 = three sets,
    one barrier; -1 only queries. Returns the previous setting."""
    return int(lib().da_gemm4w_variant(int(v)))


def _f16_cuda(t, name):
    _req(t.is_cuda, f"{name} must be on GPU")
    _req(t.dtype == torch.float16, f"{name} must be fp16, got {t.dtype}")


def gemm_f16(a, w, bias=None, epi: int = EPI_NONE, resid=None, out=None) -> torch.Tensor:
    """out = epi(a @ w^T) in fp16 (fp32 accumulate); epi NONE / BIAS / GELU / RESID."""
    _f16_cuda(a, "a"); _f16_cuda(w, "w")
    M, K = a.shape
    N = w.shape[0]
    _req(w.shape[1] == K and w.is_contiguous() and a.stride(1) == 1 and a.stride(0) % 8 == 0, "gemm_f16 layout")
    _req(K % 64 == 0 and K >= 128 and N % 8 == 0, f"gemm_f16 shape N={N} K={K}")
    _req(epi in (EPI_NONE, EPI_BIAS, EPI_GELU, EPI_RESID), "gemm_f16 epilogue")
    if bias is not None:
        _f16_cuda(bias, "bias"); _req(bias.numel() == N, "bias")
    ldr = 0
    if epi == EPI_RESID:
        _f16_cuda(resid, "resid")
        _req(resid.shape == (M, N) and resid.stride(1) == 1 and resid.stride(0) % 8 == 0, "resid")
        ldr = resid.stride(0)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float16, device=a.device)
    _req(out.dtype == torch.float16 and out.shape == (M, N) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "out")
    _check(lib().da_gemm_f16(_ptr(a), a.stride(0), _ptr(w), _ptr(out), out.stride(0), _ptr(bias), _ptr(resid), ldr,
                             M, N, K, epi, _stream()), "gemm_f16")
    return out


def flash_attn_f16(q, k, v, cu_seqlens, max_seqlen: int, H: int, Hkv: int, D: int, causal: bool = False,
                   scale: float | None = None, out=None):
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _f16_cuda(t, n)
        _req(t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0, f"{n} layout")
    _i32(cu_seqlens, "cu_seqlens")
    _req(D in (64, 96) and H % Hkv == 0, "flash_attn_f16: D 64 / 96")
    T = q.shape[0]
    if out is None:
        out = torch.empty((T, H * D), dtype=torch.float16, device=q.device)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    _check(lib().da_flash_attn_f16(_ptr(q), _ptr(k), _ptr(v), q.stride(0), k.stride(0), v.stride(0), _ptr(cu_seqlens),
                                   cu_seqlens.numel() - 1, int(max_seqlen), H, Hkv, D, int(causal), float(scale),
                                   _ptr(out), out.stride(0), _stream()), "flash_attn_f16")
    return out


def layernorm_f16(x, g, b, eps: float, resid=None, out=None):
    _f16_cuda(x, "x")
    M, D = x.shape
    _req(x.is_contiguous() and D % 8 == 0, "x must be contiguous, D % 8 == 0")
    if resid is not None:
        _f16_cuda(resid, "resid"); _req(resid.is_contiguous() and resid.shape == x.shape, "bad resid")
    _f16_cuda(g, "g"); _f16_cuda(b, "b")
    if out is None:
        out = torch.empty_like(x)
    _check(lib().da_layernorm_f16(_ptr(x), _ptr(resid), _ptr(g), _ptr(b), _ptr(out), M, D, float(eps), _stream()),
           "layernorm_f16")
    return out


def bert_embed_ln_f16(ids, positions, types, word, pos, type_, g, b, eps: float, out=None):
    _i32(ids, "ids"); _i32(positions, "positions")
    for t, n in ((word, "word"), (pos, "pos"), (type_, "type"), (g, "g"), (b, "b")):
        _f16_cuda(t, n)
    T, D = ids.numel(), word.shape[1]
    _req(positions.numel() == T and D % 8 == 0, "positions length / D")
    if out is None:
        out = torch.empty((T, D), dtype=torch.float16, device=ids.device)
    _check(lib().da_bert_embed_ln_f16(_ptr(ids), _ptr(positions), _ptr(types), _ptr(word), _ptr(pos), _ptr(type_),
                                      _ptr(g), _ptr(b), _ptr(out), T, D, float(eps), _stream()), "bert_embed_ln_f16")
    return out


def pool_l2norm_f16(h, cu_seqlens, mode: int = 0, out32=None, out16=None):
    """fp16 hidden states -> unit-norm pooled rows, fp32 and / or bf16 (the index storage type)."""
    _f16_cuda(h, "h"); _i32(cu_seqlens, "cu_seqlens")
    B, D = cu_seqlens.numel() - 1, h.shape[1]
    _req(h.is_contiguous() and D % 8 == 0, "h contiguous")
    if out16 is not None:
        _bf16_cuda(out16, "out16")
    if out32 is None and out16 is None:
        out32 = torch.empty((B, D), dtype=torch.float32, device=h.device)
    _check(lib().da_pool_l2norm_f16(_ptr(h), _ptr(cu_seqlens), B, D, mode, _ptr(out32), _ptr(out16), _stream()),
           "pool_l2norm_f16")
    return out32 if out32 is not None else out16
