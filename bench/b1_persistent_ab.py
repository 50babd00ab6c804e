"""Batch-1 decode step, full Phi-3-mini (32 layers, random init): the persistent launch
(ops/csrc/decode_b1.hip, all layers + LM head in one kernel) vs the per-kernel path (5 launches per
layer), same weights, same prompt, interleaved rounds. Prints one JSON line per round and a
summary: ms per decode step (device-synchronised decode phase / steps) and tokens equal."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models import llama as LM  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402


def main():
    L = int(os.environ.get("PROMPT", "2900"))
    steps = int(os.environ.get("STEPS", "64"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    cfg = decoder_config("phi3-mini")
    m = LM.LlamaDecoder(cfg, "cuda", seed=0)
    g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, use_graphs=True)
    prompt = [int(t) for t in np.random.default_rng(0).integers(5, 32000, size=L)]
    res = {"persistent": [], "per_kernel": []}
    toks = {}
    for r in range(rounds + 1):
        for arm, on in (("persistent", True), ("per_kernel", False)):
            LM._DECODE_B1 = on
            g.states.clear()  # re-capture the decode graph for this arm
            g.sync_phases = True
            d0, s0 = g.stats["decode_s"], g.stats["decode_steps"]
            t0 = time.perf_counter()
            out = g.generate([prompt], steps)[0]
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ms = (g.stats["decode_s"] - d0) * 1000 / max(1, g.stats["decode_steps"] - s0)
            toks[arm] = out.tokens
            if r > 0:  # round 0 = capture / warm-up
                res[arm].append(ms)
                print(json.dumps({"round": r, "arm": arm, "decode_ms_per_step": round(ms, 4),
                                  "answer_wall_ms": round(wall * 1000, 2)}), flush=True)
    LM._DECODE_B1 = False  # the library default
    print(json.dumps({"summary": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                      "tokens_equal": toks["persistent"] == toks["per_kernel"], "prompt": L, "steps": steps}))


if __name__ == "__main__":
    main()
