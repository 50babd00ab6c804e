"""Pipelined QA waves vs one wave after the other (Generator.generate_overlapped vs generate),
Phi-3-mini, B prompts of ~2.9k tokens per wave, 64 new tokens: wall time of N waves each way, plus
each phase alone on its lane (decode on the decode lane, prefill on the prefill lane) and where
the prefill moved to the full chip."""
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
from docagents_amd.ops import streams as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=2900)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--waves", type=int, default=4)
    ap.add_argument("--fracs", default="0.5")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = decoder_config("phi3-mini")
    m = LlamaDecoder(cfg, dev, seed=0)
    B = a.batch
    m.alloc_cache(2 * B + 4, 4096)
    gen = Generator(m, max_batch=B, max_seq=4096, temperature=0.2, seed=0, eos=(), share_prefix=False)
    rng = np.random.default_rng(0)
    waves = [[rng.integers(300, cfg.vocab, size=int(a.ctx + rng.integers(-50, 50))).tolist() for _ in range(B)]
             for _ in range(a.waves)]

    def seq():
        for w in waves:
            gen.generate(w, a.new)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t) * 1000, 1)
    seq()
    t_seq = min(timed(seq) for _ in range(2))
    print(json.dumps({"mode": "sequential", "waves": a.waves, "B": B, "ms": t_seq, "ms_per_wave": round(t_seq / a.waves, 1)}),
          flush=True)
    for f in [float(x) for x in a.fracs.split(",")]:
        lanes = S.lane_streams(f, dev)

        def ov():
            gen.generate_overlapped(lambda i: waves[i] if i < len(waves) else None, a.new, lanes)
        ov()
        gen.stats.pop("overlap_moves", None); gen.stats.pop("overlap_decode_join_s", None)
        t_ov = timed(ov)
        print(json.dumps({"mode": "overlapped", "frac_decode": f, "ms": t_ov, "ms_per_wave": round(t_ov / a.waves, 1),
                          "speedup": round(t_seq / t_ov, 3), "moves": gen.stats.get("overlap_moves"),
                          "decode_join_s": gen.stats.get("overlap_decode_join_s")}), flush=True)


if __name__ == "__main__":
    main()
