"""Batch-1 / small-batch decode attention in a captured graph (32 launches, like 32 layers), per
split size: us per launch (graph replay, no launch overhead). Phi-3 shape, fused RoPE, 2937 keys of
a 4096-key cache. Prints one JSON line per (B, chunk)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H, D, S, L = 32, 96, 4096, 2937
    cs = R.rope_table(S, D, 10000.0, device=dev)
    for B in (1, 4):
        kc = torch.randn(B + 1, H, S, D, device=dev).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(B, 3 * H * D, device=dev).to(torch.bfloat16)
        lens = torch.full((B,), L, dtype=torch.int32, device=dev)
        slot = torch.arange(B, dtype=torch.int32, device=dev) + 1
        for chunk in (0, 192, 256, 320, 384, 512, 768, 1024):
            out = torch.empty(B, H * D, device=dev, dtype=torch.bfloat16)
            fn = lambda: K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_len=S, chunk=chunk, rope=(cs, lens - 1), out=out)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    fn()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(32):
                    fn()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            ch, ns = K._decode_split(B, H, S, chunk)
            print(json.dumps({"B": B, "chunk_arg": chunk, "chunk": ch, "nsplit": ns,
                              "us_per_launch": round(e0.elapsed_time(e1) / 20 / 32 * 1000, 2)}), flush=True)


if __name__ == "__main__":
    main()
