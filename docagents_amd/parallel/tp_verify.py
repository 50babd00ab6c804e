"""Per-decision agreement of a tensor-parallel decoder with the unsharded one (C3 / C4 check).

Used by ``bench.py`` at N > 1 (the TP = N verdict reported next to the timed TP decode) and by the
multi-process tests (``tests/dist_checks.py``). Collective over ``group``: every rank builds the same
full model from a fixed seed, its own shard of it, and runs the same prompts.

Why per decision: random-init logits are flat AND bf16-quantised, so greedy tokens of a TP model
(partial sums reduced in another order) and the unsharded model may legitimately part at a top-1 /
top-2 tie. Teacher-forced on the unsharded model's greedy continuation, every step gives
(gap = top-1 minus top-2 logit of the unsharded model, its argmax, the TP model's argmax) and
d = the max |logit difference| over all steps and the whole vocabulary (rounding noise of the
partial sums only; a wrong-rank / stale-buffer bug is an O(1) error). A decision with gap > 2 d
cannot be flipped by that noise, so:

* ``checked`` = decisions with gap > 2 d; every one must have the same argmax (``checked_agree``);
* the free-running TP generation equals the unsharded one up to each prompt's first unchecked step
  (``prefix_ok``);
* ``wrong_order=True`` loads the neighbour's shard: the negative control, which must fail.

The reference has no TP; this pins the north star's "TP all-reduce" (C3) and the
vocab-parallel sampler (C4) to the unsharded model's decisions.
"""
from __future__ import annotations

import torch


def verdict_arch(world: int) -> str:
    """The miniature decoder the verdict runs at TP = ``world``: tiny-dec (4 heads / 2 KV heads) splits
    two ways; from three ranks the Llama-3-70B-shaped tiny-dec-tp8 (16 heads / 8 KV heads)."""
    from ..models.configs import decoder_config
    for name in ("tiny-dec", "tiny-dec-tp8"):
        c = decoder_config(name)
        if c.heads % world == 0 and c.kv_heads % world == 0 and c.ffn % (16 * world) == 0 and c.vocab % world == 0:
            return name
    raise ValueError(f"no verdict decoder splits {world} ways")


def decision_verdict(rank: int, world: int, group=None, device="cpu", arch: str | None = None,
                     wrong_order: bool = False, steps: int = 8) -> dict:
    from ..engine.generator import Generator
    from ..models.configs import decoder_config
    from ..models.llama import LlamaDecoder, TPContext, random_weights, shard_weights
    dev = torch.device(device)
    arch = arch or verdict_arch(world)
    cfg = decoder_config(arch)
    full = random_weights(cfg, dev, seed=5)
    ref = LlamaDecoder(cfg, dev, weights=full)
    src = (rank + 1) % world if wrong_order else rank
    tp = LlamaDecoder(cfg, dev, tp=TPContext(rank, world, group), weights=shard_weights(cfg, full, src, world))
    prompts = [list(range(30 + 7 * i, 30 + 7 * i + n)) for i, n in enumerate((9, 33, 4, 17, 25, 6, 40, 12))]
    a = Generator(ref, max_batch=8, max_seq=256, temperature=0.0, use_graphs=False).generate(prompts, steps)
    b = Generator(tp, max_batch=8, max_seq=256, temperature=0.0, use_graphs=False).generate(prompts, steps)

    def last_logits(m, seq):
        i32 = dict(dtype=torch.int32, device=dev)
        return m.prefill(torch.tensor(seq, **i32), torch.arange(len(seq), **i32), torch.zeros(len(seq), **i32),
                         torch.tensor([0, len(seq)], **i32), len(seq),
                         torch.tensor([len(seq) - 1], device=dev))[0].float()
    ref.alloc_cache(1, 256)
    tp.alloc_cache(1, 256)
    d, dec = 0.0, []  # dec[i] = [(gap, ref argmax, tp argmax)] per step of prompt i
    for p, x in zip(prompts, a):
        st = []
        for t in range(len(x.tokens)):
            lr, lt = last_logits(ref, p + x.tokens[:t]), last_logits(tp, p + x.tokens[:t])
            d = max(d, float((lr - lt).abs().max()))
            top = torch.topk(lr, 2)
            st.append((float(top.values[0] - top.values[1]), int(top.indices[0]), int(lt.argmax())))
        dec.append(st)
    flat = [s_ for st in dec for s_ in st]
    checked = [s_ for s_ in flat if s_[0] > 2 * d]
    agree = sum(1 for _, r_, t_ in checked if r_ == t_)
    prefix_ok, stable = [], 0
    for st, x, y in zip(dec, a, b):
        n = next((j for j, s_ in enumerate(st) if s_[0] <= 2 * d), len(st))  # first undecidable step
        stable += n == len(st)
        prefix_ok.append(x.tokens[:n] == y.tokens[:n])  # tokens[t] is the decision of step t
    xg = tp.tp.xgmi
    calls = xg.calls if xg is not None else 0
    tp.tp.close()  # collective: the verdict's communicators are not left mapped on the peers
    return {"arch": arch, "world": world, "wrong_order": wrong_order,
            "decisions": len(flat), "checked": len(checked), "checked_agree": agree,
            "prefix_ok": prefix_ok, "stable_prompts": stable, "max_logit_diff": d,
            "max_prob_diff": max(abs(x.mean_prob - y.mean_prob) for x, y in zip(a, b)),
            "xgmi": xg is not None, "xgmi_calls": calls,
            "gaps": [[round(s_[0], 4) for s_ in st] for st in dec], "tokens": [y.tokens for y in b]}


def verdict_ok(v: dict) -> bool:
    """Every rounding-proof decision agrees, they are most decisions (>= 60 %), the logit noise is
    rounding-sized, and the free-running tokens are identical up to each prompt's first undecidable
    step."""
    return (v["max_logit_diff"] < 0.05 and v["checked"] >= 0.6 * v["decisions"]
            and v["checked_agree"] == v["checked"] and all(v["prefix_ok"]) and v["max_prob_diff"] < 1e-3)
