"""Model-level numerics on the GPU: the HIP-kernel path vs the fp32-PyTorch reference path on the
same weights, plus HIP-graph decode vs eager decode."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models.bert import BertEncoder  # noqa: E402
from docagents_amd.models.configs import decoder_config, encoder_config  # noqa: E402
from docagents_amd.models.llama import LlamaDecoder, pack_prompts  # noqa: E402
from docagents_amd.ops import reference  # noqa: E402


def _to(w, dev):
    if isinstance(w, dict):
        return {k: _to(v, dev) for k, v in w.items()}
    if isinstance(w, list):
        return [_to(v, dev) for v in w]
    return w.to(dev)


def test_encoder_matches_reference():
    cfg = encoder_config("tiny-enc")
    enc = BertEncoder(cfg, "cuda", seed=3)
    ref = BertEncoder(cfg, "cuda", weights=enc.w)
    ref.ops = reference
    seqs = [list(range(5, 5 + n)) for n in (3, 70, 130, 1)]
    a = enc.encode_packed(seqs)
    b = ref.encode_packed(seqs)
    assert torch.allclose(a, b.to(a.device), atol=3e-2), (a - b).abs().max()
    cos = (a * b).sum(-1)
    assert cos.min() > 0.999


def test_decoder_prefill_matches_reference():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=1)
    m.alloc_cache(4, 512)
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(4, 512)
    prompts = [list(range(10, 10 + n)) for n in (5, 100, 33)]
    flat, pos, cu, lens = pack_prompts(prompts)
    slot_tok = np.repeat(np.arange(3, dtype=np.int32), lens)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    last = to((cu[1:] - 1).astype(np.int64))
    la = m.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    lb = r.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    assert (la.float() - lb.float()).abs().max() < 0.05
    assert torch.allclose(m.cache.buf.float(), r.cache.buf.float(), atol=0.05)


def test_generate_graph_equals_eager_greedy():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=2)
    m.alloc_cache(9, 512)
    g1 = Generator(m, max_batch=8, max_seq=512, temperature=0.0, use_graphs=True)
    prompts = [list(range(20, 20 + n)) for n in (7, 50, 3)]
    out1 = g1.generate(prompts, 12)
    m2 = LlamaDecoder(cfg, "cuda", weights=m.w)
    m2.alloc_cache(9, 512)
    g2 = Generator(m2, max_batch=8, max_seq=512, temperature=0.0, use_graphs=False)
    out2 = g2.generate(prompts, 12)
    for a, b in zip(out1, out2):
        assert a.tokens == b.tokens
        assert abs(a.mean_prob - b.mean_prob) < 1e-4
        assert len(a.tokens) == 12


def test_generate_matches_reference_greedy():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=4)
    m.alloc_cache(5, 256)
    g = Generator(m, max_batch=4, max_seq=256, temperature=0.0, use_graphs=True)
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(5, 256)
    gr = Generator(r, max_batch=4, max_seq=256, temperature=0.0, use_graphs=False)
    gr.is_cuda = False
    prompts = [list(range(40, 60)), list(range(3, 9))]
    a, b = g.generate(prompts, 6), gr.generate(prompts, 6)
    agree = sum(x == y for p, q in zip(a, b) for x, y in zip(p.tokens, q.tokens))
    assert agree >= 10  # bf16 vs fp32 may flip a near-tie late in the sequence


def test_generate_shared_prompt_head_matches_unshared():
    """Shared-head prefill (head once, suffixes vs cached head keys) and decode (every row reads the
    head's keys from the one slot holding them) generate what the plain per-prompt path generates
    (bf16: allow rare near-tie flips)."""
    m = LlamaDecoder(decoder_config("tiny-dec"), "cuda", seed=6)
    m.alloc_cache(9, 1024)
    g = Generator(m, max_batch=8, max_seq=1024, temperature=0.0, use_graphs=True)
    rng = np.random.default_rng(11)
    head = [int(t) for t in rng.integers(5, 3000, size=261)]
    prompts = [head + [int(t) for t in rng.integers(5, 3000, size=n)] for n in (1, 300, 45, 128, 9)]
    g.share_prefix = False
    want = g.generate(prompts, 12)
    g.share_prefix = True
    got = g.generate(prompts, 12)
    assert g.stats["shared_prefix_tokens"] == 256 * 4
    agree = np.mean([np.mean([x == y for x, y in zip(a.tokens, b.tokens)]) for a, b in zip(got, want)])
    assert agree >= 0.75, agree
    assert max(abs(a.mean_prob - b.mean_prob) for a, b in zip(got, want)) < 0.02


def test_continuous_scheduler_prompt_head_cache_graphs():
    """Graph-replayed continuous batching with a cached prompt head: same tokens as per-prompt runs."""
    from docagents_amd.engine.generator import ContinuousScheduler
    m = LlamaDecoder(decoder_config("tiny-dec"), "cuda", seed=8)
    m.alloc_cache(8, 1024)
    g = Generator(m, max_batch=4, max_seq=1024, temperature=0.0, use_graphs=True)
    rng = np.random.default_rng(12)
    head = [int(t) for t in rng.integers(5, 3000, size=300)]
    prompts = [head + [int(t) for t in rng.integers(5, 3000, size=n)] for n in (5, 64, 200, 17, 90)]
    g.share_prefix = False
    want = [g.generate([p], 8)[0] for p in prompts]
    g.share_prefix = True
    sched = ContinuousScheduler(g, B=4, max_new_cap=8, chunk_steps=4)
    res = sched.run_all(prompts, 8)
    assert sched.stats["heads_built"] == 1 and sched.stats["head_hits"] == 5
    agree = np.mean([np.mean([x == y for x, y in zip(a.tokens, b.tokens)]) for a, b in zip(res, want)])
    assert agree >= 0.75, agree
