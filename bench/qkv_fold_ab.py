"""Batch-64 decode step, full Phi-3-mini (32 layers, random init), ~2.9k-token prompts: the QKV
projection's split-K reduce folded into the decode attention's prologue (models/llama.py
_QKV_FOLD) vs the reduce launch, same weights, same prompts, interleaved rounds, graph-replayed.
Prints one JSON line per (round, arm) and a summary: ms per decode step (device-synchronised decode
phase / steps) and whether both arms sampled the same tokens."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models import llama as LM  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402


def main():
    L = int(os.environ.get("PROMPT", "2900"))
    B = int(os.environ.get("BATCH", "64"))
    steps = int(os.environ.get("STEPS", "32"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    m = LM.LlamaDecoder(decoder_config("phi3-mini"), "cuda", seed=0)
    g = Generator(m, max_batch=B, max_seq=4096, temperature=0.2, use_graphs=True)
    rng = np.random.default_rng(0)
    prompts = [[int(t) for t in rng.integers(5, 32000, size=L)] for _ in range(B)]
    res = {"fold": [], "reduce": []}
    toks = {}
    for r in range(rounds + 1):
        for arm, on in (("fold", True), ("reduce", False)):
            LM._QKV_FOLD = on
            g.states.clear()  # re-capture the decode graph for this arm
            g.sync_phases = True
            d0, s0 = g.stats["decode_s"], g.stats["decode_steps"]
            out = g.generate(prompts, steps)
            torch.cuda.synchronize()
            ms = (g.stats["decode_s"] - d0) * 1000 / max(1, g.stats["decode_steps"] - s0)
            toks[arm] = [o.tokens for o in out]
            if r > 0:  # round 0 = capture / warm-up
                res[arm].append(ms)
                print(json.dumps({"round": r, "arm": arm, "decode_ms_per_step": round(ms, 4)}), flush=True)
    LM._QKV_FOLD = False  # the library default
    print(json.dumps({"summary": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                      "tokens_equal": toks["fold"] == toks["reduce"], "prompt": L, "batch": B, "steps": steps}))


if __name__ == "__main__":
    main()
