"""DTYPE=fp16 encoder (BASELINE config 4 "BGE-large fp16 embedder"): the fp16 instantiations of the
phase-split GEMM (v_mfma_f32_16x16x32_f16), flash attention (32x32x16 f16), LayerNorm / embeddings /
pooling against fp32 PyTorch oracles, and the whole BGE-large-width encoder against the reference
model and against the bf16 encoder on the same weights."""
import copy
import dataclasses

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.models.bert import BertEncoder  # noqa: E402
from docagents_amd.models.configs import encoder_config  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

DEV = torch.device("cuda", 0)


def _h(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.float16)


@pytest.mark.parametrize("M,N,Kd", [(1, 1024, 1024), (77, 3072, 1024), (640, 1024, 4096), (2048, 3072, 1024),
                                    (8192, 3072, 1024)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID])
def test_gemm_f16_matches_fp32(M, N, Kd, epi):
    torch.manual_seed(M + N + epi)
    a, w = _h(M, Kd), _h(N, Kd, scale=Kd ** -0.5)
    bias = _h(N) if epi in (K.EPI_BIAS, K.EPI_GELU) else None
    r = _h(M, N) if epi == K.EPI_RESID else None
    got = K.gemm_f16(a, w, bias=bias, epi=epi, resid=r)
    ref = R.gemm_f16(a, w, bias=bias, epi=epi, resid=r)
    assert got.dtype == torch.float16
    torch.testing.assert_close(got.float(), ref.float(), atol=6e-3, rtol=6e-3)


@pytest.mark.parametrize("lens", [[128, 512, 17, 1], [300, 77]])
def test_flash_attn_f16_bidirectional_matches_fp32(lens):
    H, D = 16, 64
    T = sum(lens)
    cu = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int32, device=DEV)
    qkv = _h(T, 3 * H * D)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    got = K.flash_attn_f16(q, k, v, cu, max(lens), H, H, D)
    ref = R.flash_attn_f16(q, k, v, cu, max(lens), H, H, D)
    torch.testing.assert_close(got.float(), ref.float(), atol=4e-3, rtol=4e-3)


def test_layernorm_embed_pool_f16_match_fp32():
    T, D = 300, 1024
    x, r = _h(T, D), _h(T, D)
    g, b = (_h(D) * 0.1 + 1).to(torch.float16), _h(D, scale=0.1)
    torch.testing.assert_close(K.layernorm_f16(x, g, b, 1e-12, resid=r).float(),
                               R.layernorm_f16(x, g, b, 1e-12, resid=r).float(), atol=4e-3, rtol=4e-3)
    ids = torch.randint(0, 1000, (T,), dtype=torch.int32, device=DEV)
    pos = torch.arange(T, dtype=torch.int32, device=DEV)
    word, pe, te = _h(1000, D, scale=0.02), _h(512, D, scale=0.02), _h(2, D, scale=0.02)
    torch.testing.assert_close(K.bert_embed_ln_f16(ids, pos, None, word, pe, te, g, b, 1e-12).float(),
                               R.bert_embed_ln_f16(ids, pos, None, word, pe, te, g, b, 1e-12).float(),
                               atol=4e-3, rtol=4e-3)
    cu = torch.tensor([0, 100, 101, 300], dtype=torch.int32, device=DEV)
    for mode in (0, 1):
        torch.testing.assert_close(K.pool_l2norm_f16(x, cu, mode), R.pool_l2norm_f16(x, cu, mode).to(DEV),
                                   atol=1e-3, rtol=1e-3)


def test_bge_large_width_fp16_encoder_vs_reference_and_bf16():
    """BGE-large width (hidden 1024, 16 heads of D = 64, FFN 4096), 2 layers: the fp16 encoder on the
    kernels vs the same fp16 model on the fp32 reference ops, and vs the bf16 encoder."""
    cfg = dataclasses.replace(encoder_config("bge-large"), layers=2)
    e16 = BertEncoder(cfg, "cuda", seed=4, dtype="fp16")
    ref = BertEncoder(cfg, "cuda", weights=copy.deepcopy(e16.w), dtype="fp16")
    ref.ops = R
    seqs = [[int(t) for t in np.random.default_rng(n).integers(1000, 30000, size=n)] for n in (512, 300, 17, 1, 129)]
    a = e16.encode_packed(seqs)
    b = ref.encode_packed(seqs).to(a.device)
    cos = (a.float() * b.float()).sum(-1)
    assert cos.min() > 0.9995, cos
    wb = {k: (v.to(torch.bfloat16) if isinstance(v, torch.Tensor) else
              [{n: t.to(torch.bfloat16) for n, t in L.items()} for L in v]) for k, v in e16.w.items()}
    e_bf = BertEncoder(cfg, "cuda", weights=wb)
    c = e_bf.encode_packed(seqs)
    cos2 = (a.float() * c.float()).sum(-1)
    assert cos2.min() > 0.995, cos2
