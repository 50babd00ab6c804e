"""CPU side of the batch-1 decode's merged O projection (models/llama.py _o_merge; kernels
da_decode_attn_parts + da_gemv_omerge, GPU bit-identity in tests/test_o_merge_gpu.py): the split
partials of the fp32 oracle merge to plain softmax attention, and a decoder's batch-1 steps give
the same logits with the fold on or off."""
import dataclasses
import math

import numpy as np
import torch

from docagents_amd.models import llama as LM
from docagents_amd.models.configs import decoder_config
from docagents_amd.ops import reference as R


def test_split_partials_merge_to_softmax_attention():
    torch.manual_seed(0)
    H, Hkv, D, max_seq = 8, 4, 64, 2048
    kc = torch.randn((2, Hkv, max_seq, D)).to(torch.bfloat16)
    vc = torch.randn((2, Hkv, max_seq, D)).to(torch.bfloat16)
    q = torch.randn((1, H * D)).to(torch.bfloat16)
    slot = torch.tensor([1], dtype=torch.int32)
    assert R.decode_parts_splits(Hkv, max_seq) == 4
    for L in (1, 64, 700, 1999):
        lens = torch.tensor([L], dtype=torch.int32)
        parts = R.decode_attn_parts(q, kc, vc, lens, slot, H, Hkv, D, max_len=max_seq)
        assert parts.po.shape == (H, 4, D)
        # splits past the row's keys stay empty (max -inf, sum 0) and weigh nothing in the merge
        c = min(((L + 3) // 4 + 63) & ~63, 512)  # attention.hip dec_chunk
        assert bool(torch.isinf(parts.pm).any()) == (3 * c >= L)
        got = R.merge_parts(parts).view(H, D)
        kk = kc[1, :, :L].float().repeat_interleave(H // Hkv, 0)
        vv = vc[1, :, :L].float().repeat_interleave(H // Hkv, 0)
        p = (q.float().view(H, 1, D) @ kk.transpose(1, 2) / math.sqrt(D)).softmax(-1)
        want = (p @ vv)[:, 0]
        assert torch.allclose(got, want, atol=2e-5, rtol=1e-4), (L, (got - want).abs().max())


def test_decoder_batch1_steps_same_with_merged_o_projection():
    cfg = dataclasses.replace(decoder_config("tiny-dec-tp8"), layers=2)  # hidden 512: K % 512 == 0
    m = LM.LlamaDecoder(cfg, "cpu", seed=3)
    m.alloc_cache(2, 2048)
    assert not LM._O_MERGE  # off by default (measured no faster on the MI355X)
    logits = {}
    rng = np.random.default_rng(1)
    toks = [int(t) for t in rng.integers(5, 3000, size=4)]
    for on in (True, False):
        old = LM._O_MERGE
        LM._O_MERGE = on
        try:
            assert m._o_merge(1) == on and not m._o_merge(2)
            m.cache.buf.zero_()
            st = LM.DecodeState(m, 1, 8, 0.0, 0, ())
            st.slot.fill_(0); st.active.fill_(1); st.start.zero_()
            out = []
            for i, t in enumerate(toks):
                st.tokens.fill_(t); st.lens.fill_(i + 1); st.pos.fill_(i)
                m.decode_step(st)
                out.append(st.logits.float().clone())
            logits[on] = torch.stack(out)
        finally:
            LM._O_MERGE = old
    assert torch.allclose(logits[True], logits[False], atol=3e-2), (logits[True] - logits[False]).abs().max()


def test_split_count_rule_matches_the_kernels_module():
    """reference._decode_split mirrors kernels._decode_split (the launch's split count is what the
    O projection's merge is sized for)."""
    from docagents_amd.ops import kernels as K
    for B in (1, 2, 16, 64):
        for Hkv in (8, 32):
            for max_len in (256, 1000, 4096, 8192):
                for chunk in (0, 256, 1024):
                    assert K._decode_split(B, Hkv, max_len, chunk) == R._decode_split(B, Hkv, max_len, chunk)
    assert K.decode_parts_splits(32, 4096) == R.decode_parts_splits(32, 4096) == 8


def test_decoder_64_row_steps_same_with_qkv_fold():
    """The 33..64-row decode with the QKV reduce folded into the attention (reference stand-ins:
    the oracle keeps the finished projection) runs the same steps as the reduce-launch path."""
    cfg = dataclasses.replace(decoder_config("tiny-dec-tp8"), layers=2, heads=8, kv_heads=8)  # MHA
    m = LM.LlamaDecoder(cfg, "cpu", seed=5)
    m.alloc_cache(36, 256)
    B = 34
    assert not LM._QKV_FOLD  # off by default (measured no faster on the MI355X)
    logits = {}
    for on in (True, False):
        old = LM._QKV_FOLD
        LM._QKV_FOLD = on
        try:
            assert m._qkv_fold(B) == on and not m._qkv_fold(8)
            m.cache.buf.zero_()
            st = LM.DecodeState(m, B, 8, 0.0, 0, ())
            st.slot.copy_(torch.arange(B, dtype=torch.int32)); st.active.fill_(1); st.start.zero_()
            st.lens.fill_(1); st.pos.zero_()
            st.tokens.copy_(torch.arange(B, dtype=torch.int32) * 37 + 5)
            out = []
            for _ in range(3):
                m.decode_step(st)
                out.append(st.logits.float().clone())
            logits[on] = torch.stack(out)
        finally:
            LM._QKV_FOLD = old
    assert torch.equal(logits[True], logits[False])
