"""Where do the persistent batch-1 decode (decode_b1.hip) and the per-kernel path part ways?

Same weights, same prompt, both prefilled by their Generator (identical); then the two decode
states advance one step at a time, eager (GRAPHS=0) or by graph replay (GRAPHS=1), and after every
step the logits, the residual row, the sampled token and the new token's K/V cache rows of layer
0 / the last layer are compared bitwise. Prints one JSON line per step until the first mismatch
(+ 2 more), then a summary. Diagnostic for tests/test_decode_b1_gpu.py."""
import dataclasses
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models import llama as LM  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    graphs = os.environ.get("GRAPHS", "1") == "1"
    layers = int(os.environ.get("LAYERS", "4"))
    steps = int(os.environ.get("STEPS", "40"))
    cfg = dataclasses.replace(decoder_config("phi3-mini"), layers=layers)
    a = LM.LlamaDecoder(cfg, "cuda", seed=33)
    b = LM.LlamaDecoder(cfg, "cuda", weights=a.w)
    rng = np.random.default_rng(5)
    head = [int(t) for t in rng.integers(5, 32000, size=320)]
    prompt = (head + [int(t) for t in rng.integers(5, 32000, size=2500)])[64:]
    gens, waves = [], []
    for m, on in ((a, True), (b, False)):
        m.alloc_cache(4, 4096)
        LM._DECODE_B1 = on
        g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, seed=7, use_graphs=graphs)
        w = g._wave_begin([prompt], 64)
        if graphs:
            g._capture(w.st)
        gens.append(g)
        waves.append(w)
    torch.cuda.synchronize()
    sa, sb = waves[0].st, waves[1].st
    print(json.dumps({"graphs": graphs, "layers": layers, "prompt": len(prompt),
                      "slots": [w.slots for w in waves], "pre": [sa.pre.tolist(), sb.pre.tolist()],
                      "first_token_equal": bool(torch.equal(sa.tokens, sb.tokens))}), flush=True)
    first_bad, after = None, 0
    for step in range(steps):
        for m, st, on in ((a, sa, True), (b, sb, False)):
            LM._DECODE_B1 = on
            if graphs:
                st.graph.replay()
            else:
                m.decode_step(st)
        torch.cuda.synchronize()
        L = int(sa.lens[0])
        pos = L - 2  # the step wrote the K/V of the token at L - 2 (lens already advanced)
        rec = {"step": step, "L": L, "lens_equal": int(sa.lens[0]) == int(sb.lens[0]),
               "logits_equal": bool(torch.equal(sa.logits, sb.logits)),
               "logits_maxdiff": float((sa.logits.float() - sb.logits.float()).abs().max()),
               "x_equal": bool(torch.equal(sa.x, sb.x)),
               "token": [int(sa.tokens[0]), int(sb.tokens[0])]}
        for li in (0, layers - 1):
            ka = a.cache.k(li)[waves[0].slots[0], :, max(pos, 0)]
            kb = b.cache.k(li)[waves[1].slots[0], :, max(pos, 0)]
            va = a.cache.v(li)[waves[0].slots[0], :, max(pos, 0)]
            vb = b.cache.v(li)[waves[1].slots[0], :, max(pos, 0)]
            rec[f"kv{li}_equal"] = bool(torch.equal(ka, kb) and torch.equal(va, vb))
        rec["b1_error"] = K.decode_b1_error()
        bad = not (rec["logits_equal"] and rec["x_equal"] and rec["token"][0] == rec["token"][1])
        if first_bad is None or after < 3:
            print(json.dumps(rec), flush=True)
        if bad and first_bad is None:
            first_bad = step
        if first_bad is not None:
            after += 1
            if after > 3:
                break
    print(json.dumps({"summary": True, "first_mismatch_step": first_bad}), flush=True)


if __name__ == "__main__":
    main()
