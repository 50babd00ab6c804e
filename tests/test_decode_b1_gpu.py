"""Persistent batch-1 decode (ops/csrc/decode_b1.hip): every layer + the LM head in ONE launch, the
phase seams as device counters. Against the per-kernel path (5 launches per layer) on the same
weights: bit-identical logits for a step, identical tokens and log-probabilities over 64 sampled
steps (T = 0.2), with and without a shared prompt head, eager and graph-replayed."""
import dataclasses

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models import llama as LM  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402


def _pair(layers=4, seed=21, max_seq=4096):
    cfg = dataclasses.replace(decoder_config("phi3-mini"), layers=layers)
    a = LM.LlamaDecoder(cfg, "cuda", seed=seed)
    b = LM.LlamaDecoder(cfg, "cuda", weights=a.w)
    return a, b


class _Path:
    """Run with the persistent path on or off (off: the 5-launches-per-layer reference)."""

    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        self.old = LM._DECODE_B1
        LM._DECODE_B1 = self.on

    def __exit__(self, *exc):
        LM._DECODE_B1 = self.old


def _PerKernel():
    return _Path(False)


@pytest.fixture(autouse=True)
def _persistent_on():
    with _Path(True):  # the persistent launch is opt-in (off by default: slower on the MI355X)
        yield


def test_decode_b1_step_logits_bit_identical():
    a, b = _pair()
    a.alloc_cache(2, 4096)
    b.alloc_cache(2, 4096)
    assert a.unit_gains and a._b1_decode(1)
    prompt = [int(t) for t in np.random.default_rng(0).integers(5, 32000, size=777)]
    outs = []
    for m, persistent in ((a, True), (b, False)):
        g = Generator(m, max_batch=1, max_seq=4096, temperature=0.0, use_graphs=False)
        if persistent:
            r = g.generate([prompt], 3)
        else:
            with _PerKernel():
                r = g.generate([prompt], 3)
        outs.append(r[0])
    assert outs[0].tokens == outs[1].tokens
    # one decode step from identical states at several context lengths (split layouts: 64-key
    # splits up to 448-key ones, the new token in the first / a middle / the last split): the logits
    # must be the same bits, repeatedly (a stale hand-off shows up as an occasional mismatch)
    for rep, L in enumerate((501, 1500, 2777, 3000, 3583, 2777)):
        st = {}
        for m, persistent in ((a, True), (b, False)):
            s_ = LM.DecodeState(m, 1, 8, 0.0, 0)
            s_.tokens.fill_(1234 + rep); s_.pos.fill_(L - 1); s_.lens.fill_(L); s_.slot.fill_(1); s_.active.fill_(1)
            if persistent:
                m.decode_step(s_)
            else:
                with _PerKernel():
                    m.decode_step(s_)
            torch.cuda.synchronize()
            st[persistent] = (s_.logits.clone(), s_.x.clone(), m.cache.buf[:, :, 1, :, L - 1].clone())
        assert K.decode_b1_error() == 0
        d = (st[True][0].float() - st[False][0].float()).abs().max()
        assert torch.equal(st[True][0], st[False][0]), (L, d)
        assert torch.equal(st[True][1], st[False][1]), L
        assert torch.equal(st[True][2], st[False][2]), L  # the new token's k / v cache rows


@pytest.mark.parametrize("shared_head", [False, True])
def test_decode_b1_64_sampled_steps_identical_to_per_kernel_path(shared_head):
    a, b = _pair(seed=33)
    rng = np.random.default_rng(5)
    head = [int(t) for t in rng.integers(5, 32000, size=320)]
    prompts = [head + [int(t) for t in rng.integers(5, 32000, size=n)] for n in (2500, 900)]
    if not shared_head:
        prompts = [p[-len(p) + 64:] for p in prompts]
    res = []
    for m, persistent in ((a, True), (b, False)):
        m.alloc_cache(4, 4096)
        g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, seed=7, use_graphs=True)
        outs = []
        for p in prompts:  # batch 1, one after the other (the kept head serves the second)
            if persistent:
                outs.append(g.generate([p], 64)[0])
            else:
                with _PerKernel():
                    outs.append(g.generate([p], 64)[0])
        res.append(outs)
    assert K.decode_b1_error() == 0
    assert a._b1_ptrs is not None  # the persistent launch really ran
    for x, y in zip(*res):
        assert len(x.tokens) == 64 and x.tokens == y.tokens
        assert x.mean_prob == y.mean_prob
