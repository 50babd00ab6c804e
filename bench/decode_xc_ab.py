"""Batch-1 decode attention (Phi-3: 32 heads, D 96, 2937 keys of a 4096-key cache, fused RoPE):
splits merged through uncached memory vs through one XCD's L2 (kernels.DECODE_XC), alternating,
median us per launch; then the same for 2 / 4 rows."""
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
    H, D, S = 32, 96, 4096
    out = {"xc_probe": K.decode_xc_ok(dev)}
    for B in (1,):
        kc = torch.randn(B + 1, H, S, D, device=dev).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(B, 3 * H * D, device=dev).to(torch.bfloat16)
        lens = torch.full((B,), 2937, dtype=torch.int32, device=dev)
        slot = torch.arange(B, dtype=torch.int32, device=dev) + 1
        cs = R.rope_table(S, D, 10000.0, device=dev)
        res = {True: [], False: []}
        for rep in range(6):
            for xc in (False, True):
                K.DECODE_XC = xc
                for _ in range(20):
                    K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_len=S, rope=(cs, lens - 1))
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(200):
                    K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_len=S, rope=(cs, lens - 1))
                e1.record()
                torch.cuda.synchronize()
                res[xc].append(e0.elapsed_time(e1) / 200 * 1000)
        out[f"b{B}"] = {"uncached_us": round(statistics.median(res[False]), 2),
                        "same_xcd_us": round(statistics.median(res[True]), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
