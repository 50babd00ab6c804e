"""Batch-1 decode with the attention's split merge folded into the O projection (attention.hip
da_decode_attn_parts -> gemm.hip da_gemv_omerge) against the ticketed in-kernel merge followed by
the plain GEMV: the merged attention row and the projection must be the same bits (every workgroup
shape of the merged GEMV, MHA with fused RoPE and GQA), close to the fp32 oracle, and a decoder
must sample the same tokens with the fold on or off (eager and graph-replayed)."""
import dataclasses

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models import llama as LM  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

SHAPES = (81, 82, 161)  # waves per workgroup * 10 + rows per wave


def _setup(H, Hkv, D, max_seq, L, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    kc = torch.randn((2, Hkv, max_seq, D), generator=g, device="cuda").to(torch.bfloat16)
    vc = torch.randn((2, Hkv, max_seq, D), generator=g, device="cuda").to(torch.bfloat16)
    q = torch.randn((1, (H + 2 * Hkv) * D), generator=g, device="cuda").to(torch.bfloat16)
    wo = (torch.randn((H * D, H * D), generator=g, device="cuda") / (H * D) ** 0.5).to(torch.bfloat16)
    x = torch.randn((1, H * D), generator=g, device="cuda").to(torch.bfloat16)
    lens = torch.tensor([L], dtype=torch.int32, device="cuda")
    slot = torch.tensor([1], dtype=torch.int32, device="cuda")
    return q, kc, vc, wo, x, lens, slot


@pytest.mark.parametrize("L", [70, 513, 1500, 2935, 4000])
def test_o_merge_mha_fused_rope_bit_identical(L):
    H = Hkv = 32
    D, max_seq = 96, 4096
    q, kc, vc, wo, x, lens, slot = _setup(H, Hkv, D, max_seq, L, seed=L)
    cs = R.rope_table(max_seq, D, 10000.0).float().contiguous().cuda()
    pos = lens - 1
    rope = (cs, pos)
    assert K.decode_parts_splits(Hkv, max_seq) >= 2
    a_old = K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=max_seq, rope=rope)
    y_old = K.gemm(a_old, wo, epi=K.EPI_RESID, resid=x)
    try:
        for shape in SHAPES:
            K.lib().da_set_omerge_shape(shape)
            parts = K.decode_attn_parts(q, kc, vc, lens, slot, H, Hkv, D, max_len=max_seq, rope=rope)
            a_new = torch.empty_like(a_old)
            y_new = K.gemv_omerge(parts, wo, resid=x, attn_out=a_new)
            torch.cuda.synchronize()
            assert torch.equal(a_new, a_old), (L, shape, (a_new.float() - a_old.float()).abs().max())
            assert torch.equal(y_new, y_old), (L, shape, (y_new.float() - y_old.float()).abs().max())
    finally:
        K.lib().da_set_omerge_shape(82)
    # fp32 oracle of the same op (the reference runs the split partials + merge in PyTorch)
    kr, vr = kc.clone(), vc.clone()
    pr = R.decode_attn_parts(q, kr, vr, lens, slot, H, Hkv, D, max_len=max_seq, rope=rope)
    y_ref = R.gemv_omerge(pr, wo, resid=x)
    assert (y_ref.float() - y_old.float()).abs().max() < 0.05


@pytest.mark.parametrize("max_seq,L", [(4096, 3001), (8192, 7000)])
def test_o_merge_gqa_bit_identical(max_seq, L):
    H, Hkv, D = 32, 8, 128  # Llama-3-8B widths: K = 4096; 8192 keys -> 16 splits
    q, kc, vc, wo, x, lens, slot = _setup(H, Hkv, D, max_seq, L, seed=5)
    assert K.decode_parts_splits(Hkv, max_seq) == max_seq // 512
    qh = q[:, :H * D].contiguous()
    a_old = K.decode_attn(qh, kc, vc, lens, slot, H, Hkv, D, max_len=max_seq)
    y_old = K.gemm(a_old, wo, epi=K.EPI_RESID, resid=x)
    parts = K.decode_attn_parts(qh, kc, vc, lens, slot, H, Hkv, D, max_len=max_seq)
    y_new = K.gemv_omerge(parts, wo, resid=x)
    torch.cuda.synchronize()
    assert torch.equal(y_new, y_old), (y_new.float() - y_old.float()).abs().max()


class _Merge:
    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        self.old = LM._O_MERGE
        LM._O_MERGE = self.on

    def __exit__(self, *exc):
        LM._O_MERGE = self.old


@pytest.mark.parametrize("graphs", [False, True])
def test_o_merge_decoder_tokens_identical(graphs):
    cfg = dataclasses.replace(decoder_config("phi3-mini"), layers=3)
    a = LM.LlamaDecoder(cfg, "cuda", seed=41)
    b = LM.LlamaDecoder(cfg, "cuda", weights=a.w)
    rng = np.random.default_rng(9)
    prompt = [int(t) for t in rng.integers(5, 32000, size=1800)]
    res = []
    for m, on in ((a, True), (b, False)):
        m.alloc_cache(2, 4096)
        with _Merge(on):
            assert m._o_merge(1) == on
            g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, seed=3, use_graphs=graphs)
            res.append(g.generate([prompt], 48)[0])
    assert len(res[0].tokens) == 48 and res[0].tokens == res[1].tokens
    assert res[0].mean_prob == res[1].mean_prob
