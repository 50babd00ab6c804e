"""Decode-step timing of the production decoder (Phi-3-mini by default): prefill B prompts of L
tokens, then generate ``--new`` tokens through the HIP-graph decode path, ``--reps`` times.
Prints ms per decode step; run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split
(the p50 cache-miss query is B=1, the flagship batch B=64)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.models.llama import LlamaDecoder  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()  # DA_* schedule overrides for A/B sweeps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="phi3-mini")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=2870)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = decoder_config(a.arch)
    m = LlamaDecoder(cfg, dev, seed=0)
    gen = Generator(m, max_batch=max(a.batch, 1), max_seq=4096, temperature=0.2, seed=0, eos=())
    rng = np.random.default_rng(0)
    prompts = [list(rng.integers(100, cfg.vocab - 100, size=a.prompt)) for _ in range(a.batch)]
    gen.generate(prompts, a.new)  # capture + warm
    torch.cuda.synchronize()
    out = []
    for _ in range(a.reps):
        gen.sync_phases = True
        d0, s0 = gen.stats["decode_s"], gen.stats["decode_steps"]
        p0 = gen.stats.get("prefill_wall_s", 0.0)
        t = time.perf_counter()
        gen.generate(prompts, a.new)
        torch.cuda.synchronize()
        tot = time.perf_counter() - t
        steps = gen.stats["decode_steps"] - s0
        out.append({"total_ms": round(tot * 1e3, 2), "prefill_ms": round((gen.stats["prefill_wall_s"] - p0) * 1e3, 2),
                    "decode_ms_per_step": round((gen.stats["decode_s"] - d0) * 1e3 / max(1, steps), 3)})
    print(json.dumps({"arch": a.arch, "batch": a.batch, "prompt": a.prompt, "new": a.new, "runs": out}), flush=True)


if __name__ == "__main__":
    main()
