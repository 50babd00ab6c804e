"""Where do two batch-1 decode arms part ways? An arm is (path, mode): path b1 = the persistent
launch (decode_b1.hip), pk = the per-kernel path; mode e = eager decode_step calls, g = HIP-graph
replay. Same weights, same prompt, each arm prefilled by its own Generator into its own cache; then
both advance one step at a time and after every step the logits, the residual row, the sampled
token and the new token's K/V rows of the first / last layer are compared bitwise. One JSON line
per step until the first mismatch (+ 3 more), then a summary.

ARMS="b1e:pke" (default), e.g. "b1e:b1e" (is the persistent path deterministic?), "pke:pke",
"b1g:b1e". Diagnostic for tests/test_decode_b1_gpu.py."""
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


def run(arms: list[str], layers: int, steps: int):
    cfg = dataclasses.replace(decoder_config("phi3-mini"), layers=layers)
    base = LM.LlamaDecoder(cfg, "cuda", seed=33)
    models = [base, LM.LlamaDecoder(cfg, "cuda", weights=base.w)]
    rng = np.random.default_rng(5)
    head = [int(t) for t in rng.integers(5, 32000, size=320)]
    prompt = (head + [int(t) for t in rng.integers(5, 32000, size=2500)])[64:]
    sts, slots = [], []
    for m, arm in zip(models, arms):
        m.alloc_cache(4, 4096)
        LM._DECODE_B1 = arm.startswith("b1")
        g = Generator(m, max_batch=1, max_seq=4096, temperature=0.2, seed=7, use_graphs=arm.endswith("g"))
        w = g._wave_begin([prompt], 64)
        if arm.endswith("g"):
            g._capture(w.st)
        sts.append(w.st)
        slots.append(w.slots[0])
    torch.cuda.synchronize()
    print(json.dumps({"arms": arms, "layers": layers, "prompt": len(prompt), "slots": slots,
                      "b1_error_after_setup": K.decode_b1_error(),
                      "first_token_equal": bool(torch.equal(sts[0].tokens, sts[1].tokens))}), flush=True)
    first_bad, after = None, 0
    for step in range(steps):
        for m, st, arm in zip(models, sts, arms):
            LM._DECODE_B1 = arm.startswith("b1")
            if arm.endswith("g"):
                st.graph.replay()
            else:
                m.decode_step(st)
        torch.cuda.synchronize()
        sa, sb = sts
        L = int(sa.lens[0])
        pos = L - 2  # the step wrote the K/V of the token at L - 2 (lens already advanced)
        rec = {"step": step, "L": L, "lens_equal": int(sa.lens[0]) == int(sb.lens[0]),
               "logits_equal": bool(torch.equal(sa.logits, sb.logits)),
               "logits_maxdiff": float((sa.logits.float() - sb.logits.float()).abs().max()),
               "x_equal": bool(torch.equal(sa.x, sb.x)),
               "token": [int(sa.tokens[0]), int(sb.tokens[0])]}
        for li in (0, layers - 1):
            kv = [(m.cache.k(li)[s, :, pos], m.cache.v(li)[s, :, pos]) for m, s in zip(models, slots)]
            rec[f"kv{li}_equal"] = bool(torch.equal(kv[0][0], kv[1][0]) and torch.equal(kv[0][1], kv[1][1]))
        # every layer's cache rows [0, L - 1): the first (layer, position, k|v) that differs
        diff = None
        for li in range(layers):
            for nm in ("k", "v"):
                ra = getattr(models[0].cache, nm)(li)[slots[0], :, :L - 1]
                rb = getattr(models[1].cache, nm)(li)[slots[1], :, :L - 1]
                ne = (ra != rb).any(dim=-1).any(dim=0).nonzero()
                if ne.numel() and diff is None:
                    diff = {"layer": li, "which": nm, "pos": int(ne[0]), "npos": int(ne.numel())}
        rec["cache_first_diff"] = diff
        rec["qkv_equal"] = bool(torch.equal(sa.qkv, sb.qkv))
        rec["attn_equal"] = bool(torch.equal(sa.attn, sb.attn))  # the last layer's attention output
        if not rec["attn_equal"]:
            dh = (sa.attn.view(-1, cfg.head_dim) != sb.attn.view(-1, cfg.head_dim)).any(dim=1).nonzero().flatten()
            rec["attn_heads_diff"] = dh.tolist()
            rec["attn_maxdiff"] = float((sa.attn.float() - sb.attn.float()).abs().max())
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
    print(json.dumps({"summary": True, "arms": arms, "first_mismatch_step": first_bad}), flush=True)
    LM._DECODE_B1 = False  # the library default
    K.decode_b1_error(reset=True)


def main():
    layers = int(os.environ.get("LAYERS", "4"))
    steps = int(os.environ.get("STEPS", "40"))
    for pair in os.environ.get("ARMS", "b1e:pke").split(","):
        run(pair.split(":"), layers, steps)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
