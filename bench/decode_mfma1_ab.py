"""Batch-1 MHA decode attention, VALU kernel vs MFMA kernel (DA_DECODE_MFMA1=0 / 1, one process
each): 32 launches in one captured graph, each on its OWN KV cache (32 x 2 x 50 MB: HBM, not the
MALL, like 32 layers), Phi-3 shape (32 heads, D 96, 2937 keys of a 4096-key cache), no RoPE and
with the fused RoPE (that form stays on the VALU kernel). us per launch, median of 5 timings."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H, D, S, L, NL = 32, 96, 4096, 2937, 32
    B = int(os.environ.get("B", "1"))
    cs = R.rope_table(S, D, 10000.0, device=dev)
    caches = [(torch.randn(B + 1, H, S, D, device=dev).to(torch.bfloat16),
               torch.randn(B + 1, H, S, D, device=dev).to(torch.bfloat16)) for _ in range(NL)]
    q = torch.randn(B, 3 * H * D, device=dev).to(torch.bfloat16)
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    slot = torch.arange(B, dtype=torch.int32, device=dev) + 1
    out = torch.empty(B, H * D, device=dev, dtype=torch.bfloat16)
    res = {"mfma1": os.environ.get("DA_DECODE_MFMA1", "1"), "B": B}
    for rope in (False, True):
        def fn():
            for kc, vc in caches:
                K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_len=S, out=out,
                              rope=(cs, lens - 1) if rope else None)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 / NL * 1000)
        res["rope" if rope else "plain"] = round(statistics.median(ts), 2)
    # numerics of this process's kernel vs the fp32 reference (plain)
    kc, vc = caches[0]
    got = K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_len=S)
    ref = R.decode_attn(q, kc, vc, lens, slot, H, H, D)
    res["max_err"] = round(float((got.float() - ref.float()).abs().max()), 5)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
