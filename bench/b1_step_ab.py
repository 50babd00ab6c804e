"""Batch-1 answer latency A/B in one process (Phi-3-mini real dims, random weights, a 2.9k-token
prompt, 64 new tokens, Generator.generate as the engine runs it): the chunked small-batch sampler
(kernels.SAMPLE_CHUNKED_MAX_B = 64) vs one workgroup per row (0), interleaved rounds; ms per answer.
(A multi-step decode graph arm — 4 steps per replay — measured 0.7 ms SLOWER per answer and was
dropped: profiles/r3/b1_step_ab.txt.)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.models.llama import LlamaDecoder  # noqa: E402
from docagents_amd.engine.generator import Generator  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = decoder_config("phi3-mini")
    m = LlamaDecoder(cfg, dev, seed=0)
    m.alloc_cache(8, 4096)
    rng = np.random.default_rng(0)
    prompt = rng.integers(300, cfg.vocab, size=2900).tolist()
    arms = {"base": 0, "chunked_sampler": 64}
    gens = {name: Generator(m, max_batch=1, max_seq=4096, temperature=0.2, seed=3, eos=()) for name in arms}
    res = {k: [] for k in arms}
    toks = {}
    for rnd in range(6):
        for name, cb in arms.items():
            K.SAMPLE_CHUNKED_MAX_B = cb
            g = gens[name]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = g.generate([prompt], 64)
            torch.cuda.synchronize()
            if rnd > 0:
                res[name].append((time.perf_counter() - t0) * 1e3)
            toks[name] = out[0].tokens
    K.SAMPLE_CHUNKED_MAX_B = 64
    same = all(t == toks["base"] for t in toks.values())
    print(json.dumps({"ms_per_answer_median": {k: round(float(np.median(v)), 2) for k, v in res.items()},
                      "ms_per_answer_min": {k: round(float(np.min(v)), 2) for k, v in res.items()},
                      "same_tokens": same}), flush=True)


if __name__ == "__main__":
    main()
