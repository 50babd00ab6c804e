"""Batch-1 decode attention, 4 vs 8 waves per workgroup (da_set_decode_w8; w8_1tile = one tile per
wave, da_set_decode_w8_var(1)): Phi-3 shape (32 heads,
D=96, fused RoPE + new-token KV write, splits fixed by the 4096-key capacity), 32 layers' launches
over 32 distinct caches in one HIP graph; us per launch at several context lengths, optionally with
other keys-per-split caps (CHUNKS). Prints one JSON line per length."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402


def main():
    dev = torch.device("cuda")
    H, D, S, layers = 32, 96, 4096, 32
    torch.manual_seed(0)
    kcs = [torch.randn(2, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(layers)]
    vcs = [torch.randn(2, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(layers)]
    qkv = torch.randn(1, 3 * H * D, device=dev, dtype=torch.bfloat16)
    cs = R.rope_table(S, D, 10000.0).to(dev)
    slot = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(1, H * D, device=dev, dtype=torch.bfloat16)
    arms = [("w4", 0, 0), ("w8", 32, 0), ("w8_1tile", 32, -1)] + \
        [(f"w8_c{c}", 32, int(c)) for c in os.environ.get("CHUNKS", "").split(",") if c]
    for L in [int(x) for x in os.environ.get("LENS", "512,1500,2935,4000").split(",")]:
        lens = torch.full((1,), L, dtype=torch.int32, device=dev)
        pos = lens - 1
        res, outs = {"L": L}, {}
        for rnd in range(2):  # interleaved rounds
            for tag, w8, chunk in arms:
                K.lib().da_set_decode_w8(w8)
                K.lib().da_set_decode_w8_var(1 if chunk < 0 else 0)  # -1: the one-tile-per-wave variant
                chunk = max(chunk, 0)

                def run():
                    for li in range(layers):
                        K.decode_attn(qkv, kcs[li], vcs[li], lens, slot, H, H, D, max_len=S, out=out,
                                      rope=(cs, pos), chunk=chunk)
                run()
                torch.cuda.synchronize()
                outs[tag] = out.float().clone()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    run()
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    g.replay()
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1000 / 20 / layers
                res[f"{tag}_us"] = min(res.get(f"{tag}_us", 1e9), round(us, 2))
        for tag, *_ in arms:
            res[f"{tag}_TBps"] = round(2 * H * L * D * 2 / res[f"{tag}_us"] / 1e6, 2)
        res["maxdiff_vs_w4"] = max(float((o - outs["w4"]).abs().max()) for o in outs.values())
        K.lib().da_set_decode_w8(0)
        K.lib().da_set_decode_w8_var(0)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
