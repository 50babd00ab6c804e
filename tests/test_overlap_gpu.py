"""Pipelined QA waves (Generator.generate_overlapped): the decode of wave i on a CU-masked lane
beside the prefill of wave i + 1, which moves to the full chip once that decode is done. Every
wave's tokens, logprob confidences and token counts must equal the one-wave-at-a-time path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.models.llama import LlamaDecoder  # noqa: E402
from docagents_amd.ops import streams as S  # noqa: E402


@pytest.mark.parametrize("arch,n,plen", [("tiny-dec", 8, 300), ("phi3-mini", 4, 700)])
def test_overlapped_waves_match_sequential(arch, n, plen):
    dev = torch.device("cuda", 0)
    cfg = decoder_config(arch)
    m = LlamaDecoder(cfg, dev, seed=0)
    m.alloc_cache(2 * n + 4, 2048)
    gen = Generator(m, max_batch=n, max_seq=2048, temperature=0.2, seed=3, eos=())
    rng = np.random.default_rng(0)
    waves = [[rng.integers(300, cfg.vocab, size=int(plen + rng.integers(-40, 40))).tolist() for _ in range(n)]
             for _ in range(4)]
    max_new = 24
    ref = [gen.generate(w, max_new) for w in waves]
    lanes = S.lane_streams(0.5, dev)
    got = gen.generate_overlapped(lambda i: waves[i] if i < len(waves) else None, max_new, lanes)
    torch.cuda.synchronize()
    assert len(got) == len(ref)
    for r, g in zip(ref, got):
        assert [x.tokens for x in r] == [x.tokens for x in g]
        assert [x.n_tokens for x in r] == [x.n_tokens for x in g]
        np.testing.assert_allclose([x.mean_prob for x in r], [x.mean_prob for x in g], rtol=0, atol=0)
    # every slot came back
    assert len(gen.cache.free) >= 2 * n
