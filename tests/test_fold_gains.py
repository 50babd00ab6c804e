"""RMSNorm-gain folding (LlamaDecoder._fold_norm_gains): W diag(g) with g = 1 is the same model as
(W, g). A checkpoint's non-unit gains are folded at construction; the folded model's logits must
match an unfolded model's on the same weights (fp32 reference ops on the CPU; the GPU test in
test_models_gpu.py covers the fused batch-1 GEMV path that relies on the unit gain)."""
import copy

import torch

from docagents_amd.models.configs import decoder_config
from docagents_amd.models.llama import LlamaDecoder, random_weights


class _Unfolded(LlamaDecoder):
    def _fold_norm_gains(self):
        pass


def _gains(w, seed):
    g = torch.Generator().manual_seed(seed)
    for L in w["layers"]:
        for k in ("ln_attn", "ln_mlp"):
            L[k] = (0.5 + torch.rand(L[k].shape, generator=g)).to(L[k].dtype)
    w["norm"] = (0.5 + torch.rand(w["norm"].shape, generator=g)).to(w["norm"].dtype)
    return w


def _last_logits(m, seq):
    t = torch.tensor(seq, dtype=torch.int32)
    return m.prefill(t, torch.arange(len(seq), dtype=torch.int32), torch.zeros(len(seq), dtype=torch.int32),
                     torch.tensor([0, len(seq)], dtype=torch.int32), len(seq),
                     torch.tensor([len(seq) - 1]))[0].float()


def test_folded_gains_match_unfolded_model():
    cfg = decoder_config("tiny-dec")
    w = _gains(random_weights(cfg, "cpu", seed=11), seed=3)
    ref = _Unfolded(cfg, "cpu", weights=copy.deepcopy(w))
    m = LlamaDecoder(cfg, "cpu", weights=copy.deepcopy(w))
    for L in m.w["layers"]:
        assert bool((L["ln_attn"] == 1).all()) and bool((L["ln_mlp"] == 1).all())
    assert bool((m.w["norm"] == 1).all())
    assert not torch.equal(m.w["lm_head"], w["lm_head"])
    for mm in (ref, m):
        mm.alloc_cache(2, 128)
    seq = list(range(17, 17 + 40))
    a, b = _last_logits(ref, seq), _last_logits(m, seq)
    # the folded weights are rounded to bf16 once: noise of a few bf16 ulps on O(1) logits
    assert float((a - b).abs().max()) < 0.05 * max(1.0, float(a.abs().max()))
    assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) > 0.999


def test_fused_norm_prefill_matches_unfused_on_cpu(monkeypatch):
    """>= 640 tokens: the prefill folds the RMSNorms after layer 0 into the projections
    (reference.gemm8p_norm, the fp32 twin of gemm.hip da_gemm8p_norm); same logits and KV cache
    as the rmsnorm -> gemm path, on folded non-unit gains."""
    import docagents_amd.models.llama as llama
    monkeypatch.setattr(llama, "_PREFILL_NORM_FUSE", True)
    cfg = decoder_config("tiny-dec")
    w = _gains(random_weights(cfg, "cpu", seed=12), seed=4)
    m = LlamaDecoder(cfg, "cpu", weights=copy.deepcopy(w))
    u = LlamaDecoder(cfg, "cpu", weights=copy.deepcopy(w))
    u._prefill_norms_fusable = lambda T: False
    seq = [(7 * i) % 30000 + 5 for i in range(700)]
    assert m._prefill_norms_fusable(len(seq)) and not u._prefill_norms_fusable(len(seq))
    for mm in (m, u):
        mm.alloc_cache(1, 1024)
    a, b = _last_logits(m, seq), _last_logits(u, seq)
    assert float((a - b).abs().max()) < 0.05 * max(1.0, float(a.abs().max()))
    assert torch.allclose(m.cache.buf.float(), u.cache.buf.float(), atol=0.05)


def test_reference_gemm8p_norm_sums():
    """reference.gemm8p_norm EPI_RESID writes [M][N / 64] sums of squares of the bf16 rows."""
    from docagents_amd.ops import reference as R
    g = torch.Generator().manual_seed(1)
    M, N, Kd = 5, 256, 128
    a = torch.randn(M, Kd, generator=g).bfloat16()
    w = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).bfloat16()
    x = torch.randn(M, N, generator=g).bfloat16()
    ssq = torch.empty((N // 64) * M)
    y = R.gemm8p_norm(a, w, R.EPI_RESID, resid=x, ssq_out=ssq)
    assert torch.equal(y, R.gemm(a, w, epi=R.EPI_RESID, resid=x))
    ref = y.float().view(M, N // 64, 64).pow(2).sum(-1)
    assert torch.allclose(ssq.view(M, N // 64), R.gemm8p_ssq_parts(y))
    assert torch.allclose(ssq.view(M, N // 64).sum(1), ref.sum(1))
    inv = torch.rsqrt(ref.sum(1) / N + 1e-5)
    z = R.gemm8p_norm(y, w[:, :].repeat(1, 2)[:, :N], R.EPI_NONE, norm_in=(ssq, N // 64, 1e-5))
    z_ref = ((y.float() * inv[:, None]) @ w.repeat(1, 2)[:, :N].float().t()).bfloat16()
    assert torch.allclose(z.float(), z_ref.float(), atol=2e-2)
