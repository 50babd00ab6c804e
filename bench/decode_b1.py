"""Batch-1 decode attention as the decode step runs it (Phi-3: 32 heads, D=96, fused RoPE + new-token
KV write, split count fixed by the 4096-key cache capacity): 32 layers' launches over 32 distinct
caches (1.15 GB, beyond the MALL) captured in one HIP graph and replayed; us per launch for
balanced vs fixed keys per split (da_set_decode_balance) at several context lengths."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402
from ab_arms import apply_env_overrides  # noqa: E402
apply_env_overrides()


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
    for L in [int(x) for x in os.environ.get("LENS", "512,1500,2935,4000").split(",")]:
        lens = torch.full((1,), L, dtype=torch.int32, device=dev)
        pos = lens - 1
        res = {"L": L}
        outs = {}
        arms = [(0, 0), (1, 0)] + [(1, int(c)) for c in os.environ.get("CHUNKS", "").split(",") if c]
        for bal, chunk in arms:
            K.lib().da_set_decode_balance(bal)
            tag = f"bal{bal}" + (f"_c{chunk}" if chunk else "")

            def run():
                for li in range(layers):
                    K.decode_attn(qkv, kcs[li], vcs[li], lens, slot, H, H, D, max_len=S, out=out, rope=(cs, pos),
                                  chunk=chunk)
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
            for _ in range(10):
                g.replay()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1000 / 10 / layers
            res[f"{tag}_us"] = round(us, 2)
            res[f"{tag}_TBps"] = round(2 * H * L * D * 2 / us / 1e6, 2)
        res["maxdiff"] = max(float((o - outs["bal0"]).abs().max()) for o in outs.values())
        K.lib().da_set_decode_balance(1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
