"""Batch-1 decode step, full Phi-3-mini (32 layers, random init): the decode attention's split merge
folded into the O projection (models/llama.py _O_MERGE: da_decode_attn_parts + da_gemv_omerge) vs
the ticketed in-kernel merge + plain GEMV, and the merged GEMV's workgroup shapes (SHAPES, waves per
workgroup * 10 + rows per wave). Same weights, same prompt, interleaved rounds, graph-replayed.
Prints one JSON line per (round, arm) and a summary: ms per decode step (device-synchronised decode
phase / steps) and whether every arm sampled the same tokens."""
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
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    L = int(os.environ.get("PROMPT", "2900"))
    steps = int(os.environ.get("STEPS", "64"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    shapes = [int(s) for s in os.environ.get("SHAPES", "161").split(",")]
    m = LM.LlamaDecoder(decoder_config("phi3-mini"), "cuda", seed=0)
    g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, use_graphs=True)
    prompt = [int(t) for t in np.random.default_rng(0).integers(5, 32000, size=L)]
    arms = ([("ticket", False, 161)] if os.environ.get("TICKET", "1") == "1" else []) + \
        [(f"merge{s}", True, s) for s in shapes if s > 0]
    res = {a[0]: [] for a in arms}
    toks = {}
    for r in range(rounds + 1):
        for arm, on, shape in arms:
            LM._O_MERGE = on
            K.lib().da_set_omerge_shape(shape)
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
    LM._O_MERGE = True  # the library default
    K.lib().da_set_omerge_shape(82)
    print(json.dumps({"summary": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                      "tokens_equal": len({tuple(t) for t in toks.values()}) == 1, "prompt": L, "steps": steps}))


if __name__ == "__main__":
    main()
