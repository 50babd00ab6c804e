"""Probe: co-running a decode wave and a prefill wave of Phi-3-mini on complementary CU-masked
streams (ops/streams.py). Decides the decode lane's CU share for the serving pipeline.

1. placement: which XCD / CU the workgroups of a single-CU-bit stream land on (the mask bit ->
   XCD mapping), and how a lane split spreads over the XCDs;
2. for each decode share f: decode (B rows, 63 graph-replayed steps at ~2.9k context) alone on
   its f-share lane, prefill (B prompts of ~2.9k tokens) alone on the complementary lane, both
   issued together, and the same on unmasked streams. Prints one JSON line per configuration.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.ops import h2d  # noqa: E402
from docagents_amd.models.configs import decoder_config  # noqa: E402
from docagents_amd.models.llama import DecodeState, LlamaDecoder  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import streams as S  # noqa: E402


def emit(d, out):
    print(json.dumps(d), flush=True)
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(d) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ctx", type=int, default=2900)
    ap.add_argument("--steps", type=int, default=63)
    ap.add_argument("--fracs", default="0.125,0.1875,0.25,0.3125,0.375")
    ap.add_argument("--llm", default="phi3-mini")
    ap.add_argument("--skip-placement", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--expand", action="store_true", help="co-run, then move the prefill to the full chip")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_cu = S.cu_count(dev)
    emit({"cu_count": n_cu}, a.out)

    if not a.skip_placement:
        for bit in (0, 1, 2, 7, 8, 32):
            s = S.masked_stream([bit], dev)
            pl = S.probe_placement(s, blocks=64, spin=2000)
            emit({"bit": bit, "placements": sorted(set(pl))}, a.out)
        for f in (0.25,):
            la, lb = S.lane_streams(f, dev)
            for name, s in (("A", la), ("B", lb)):
                pl = S.probe_placement(s, blocks=2048, spin=20000)
                per_xcc = collections.Counter(x for x, *_ in set(pl))
                emit({"lane": name, "frac_a": f, "distinct_cus": len(set(pl)), "per_xcc": dict(sorted(per_xcc.items()))},
                     a.out)

    cfg = decoder_config(a.llm)
    m = LlamaDecoder(cfg, dev, seed=0)
    B = a.batch
    m.alloc_cache(2 * B + 2, 4096)
    gen = Generator(m, max_batch=B, max_seq=4096, temperature=0.2, seed=0, eos=(), share_prefix=False)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(300, cfg.vocab, size=int(a.ctx + rng.integers(-50, 50))).tolist() for _ in range(B)]
    max_new = a.steps + 1
    st_dec = DecodeState(m, B, max_new, 0.2, 0, ())
    st_pf = DecodeState(m, B, max_new, 0.2, 0, ())
    slots_dec = gen.cache.acquire(B)
    slots_pf = gen.cache.acquire(B)

    def init_state(st, slots):
        plen = np.asarray([len(p) for p in prompts], dtype=np.int32)
        st.pos.copy_(h2d(plen - 1, dev)); st.lens.copy_(h2d(plen, dev))
        st.slot.copy_(h2d(np.asarray(slots, dtype=np.int32), dev)); st.active.fill_(1)
        st.start.copy_(h2d(plen - 1, dev)); st.tokens.zero_(); st.hist.fill_(-1); st.conf.zero_()
        st.pre.zero_()

    init_state(st_dec, slots_dec)
    gen._prefill_into(st_dec, prompts, slots_dec, 0)
    torch.cuda.synchronize()
    gen._capture(st_dec)
    names = ("tokens", "pos", "lens", "active", "hist", "conf", "start")
    saved = {n: getattr(st_dec, n).clone() for n in names}

    def reset_dec():
        for n in names:
            getattr(st_dec, n).copy_(saved[n])

    def decode(stream):
        with torch.cuda.stream(stream):
            for _ in range(a.steps):
                st_dec.graph.replay()

    def prefill(stream):
        with torch.cuda.stream(stream), K.workspace_role("prefill"):
            init_state(st_pf, slots_pf)
            gen._prefill_into(st_pf, prompts, slots_pf, 0)

    def timed(fn):
        reset_dec()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1000

    full = torch.cuda.current_stream()
    p1, p2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):
        timed(lambda: decode(full)); timed(lambda: prefill(full))
    td = min(timed(lambda: decode(full)) for _ in range(2))
    tp = min(timed(lambda: prefill(full)) for _ in range(2))
    tc = min(timed(lambda: (decode(p1), prefill(p2))) for _ in range(2))
    emit({"mode": "unmasked", "decode_ms": round(td, 1), "prefill_ms": round(tp, 1), "concurrent_ms": round(tc, 1),
          "serial_ms": round(td + tp, 1), "B": B, "ctx": a.ctx, "steps": a.steps}, a.out)
    # co-run, then expand: the prefill starts on lane B beside the decode on lane A; before each
    # layer it checks (host side, at most two layers issued ahead) whether the decode is done and
    # then moves the rest of the prefill to a full-chip stream
    def corun_expand(sa, sb):
        done = torch.cuda.Event()
        decode(sa)
        done.record(sa)
        evs = []
        state = {"moved": False}

        def hook(li):
            if state["moved"]:
                return
            if len(evs) >= 2:
                evs[-2].synchronize()
            if done.query():
                full.wait_stream(sb)
                torch.cuda.set_stream(full)
                state["moved"] = li
                return
            ev = torch.cuda.Event()
            ev.record(sb)
            evs.append(ev)
        m.layer_hook = hook
        try:
            with torch.cuda.stream(sb), K.workspace_role("prefill"):
                init_state(st_pf, slots_pf)
                gen._prefill_into(st_pf, prompts, slots_pf, 0)
        finally:
            m.layer_hook = None
        return state["moved"]

    for f in [float(x) for x in a.fracs.split(",")]:
        sa, sb = S.lane_streams(f, dev)
        if a.expand:
            timed(lambda: decode(sa)); timed(lambda: prefill(sb))
            tdm = min(timed(lambda: decode(sa)) for _ in range(2))
            tpm = min(timed(lambda: prefill(sb)) for _ in range(2))
            moved = []
            te = min(timed(lambda: moved.append(corun_expand(sa, sb))) for _ in range(3))
            emit({"mode": "corun_expand", "frac_decode": f, "decode_masked_ms": round(tdm, 1),
                  "prefill_masked_ms": round(tpm, 1), "corun_expand_ms": round(te, 1), "moved_at_layer": moved,
                  "decode_full_ms": round(td, 1), "prefill_full_ms": round(tp, 1), "serial_full_ms": round(td + tp, 1),
                  "speedup_vs_serial": round((td + tp) / te, 3)}, a.out)
            continue
        timed(lambda: decode(sa)); timed(lambda: prefill(sb))
        tdm = min(timed(lambda: decode(sa)) for _ in range(2))
        tpm = min(timed(lambda: prefill(sb)) for _ in range(2))
        timed(lambda: (decode(sa), prefill(sb)))
        tc1 = min(timed(lambda: (decode(sa), prefill(sb))) for _ in range(2))
        tc2 = min(timed(lambda: (prefill(sb), decode(sa))) for _ in range(2))
        emit({"mode": "cumask", "frac_decode": f, "decode_masked_ms": round(tdm, 1), "prefill_masked_ms": round(tpm, 1),
              "concurrent_dec_first_ms": round(tc1, 1), "concurrent_pf_first_ms": round(tc2, 1),
              "decode_full_ms": round(td, 1), "prefill_full_ms": round(tp, 1), "serial_full_ms": round(td + tp, 1),
              "speedup_vs_serial": round((td + tp) / min(tc1, tc2), 3)}, a.out)


if __name__ == "__main__":
    main()
