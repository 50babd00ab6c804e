"""Timeline of one batch-1 decode-attention launch (Phi-3: 32 heads, D=96, fused RoPE, last-split
merge): every workgroup stamps the wall clock (100 MHz) at its start, after the prologue (q RoPE
into LDS), after its first 64-key tile, after its last tile, after storing its split partial, and at
its end (after the ticket / merge). Prints per-stage quantiles relative to the launch's first
stamp, the critical (last-finishing) workgroup, and the XCD spread of each head's splits."""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=2944)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H = Hkv = 32
    D, S, B = 96, 4096, a.batch
    torch.manual_seed(0)
    kc = torch.randn(B + 1, Hkv, S, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(B + 1, Hkv, S, D, device=dev).to(torch.bfloat16)
    qkv = torch.randn(B, (H + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    lens = torch.full((B,), a.len, device=dev, dtype=torch.int32)
    pos = lens - 1
    slot = torch.arange(B, device=dev, dtype=torch.int32)
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
    ang = torch.arange(S, dtype=torch.float32)[:, None] * inv[None]
    cs = torch.stack([ang.cos(), ang.sin()], -1).contiguous().to(dev)

    def run():
        return K.decode_attn(qkv, kc, vc, lens, slot, H, Hkv, D, max_len=S, chunk=a.chunk, rope=(cs, pos))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1000
    chunk = a.chunk
    if chunk <= 0:
        want = S * B * Hkv / 768
        chunk = 512
        while chunk < want and chunk < 4096:
            chunk *= 2
    nsplit = math.ceil(S / chunk)
    tr = torch.zeros(B * Hkv * nsplit * 16, dtype=torch.int64, device=dev)
    K.lib().da_set_decode_trace(K._ptr(tr))
    try:
        run()
        torch.cuda.synchronize()
    finally:
        K.lib().da_set_decode_trace(None)
    t = tr.view(B, Hkv, nsplit, 16).cpu().numpy()
    t0 = t[..., 0].min()
    rel = (t[..., [0, 1, 7, 2, 8, 9, 10, 11, 12, 3, 4]] - t0) * 0.01  # 100 MHz -> us
    names = ["start", "prologue", "tile1", "tiles", "w0", "w1", "w2", "w3", "merged", "stored", "end"]
    q = {n: [round(float(np.percentile(rel[..., i], p)), 2) for p in (0, 50, 100)] for i, n in enumerate(names)}
    nonempty = np.arange(nsplit)[None, None, :] * chunk < lens.cpu().numpy()[:, None, None]
    nonempty = np.broadcast_to(nonempty, rel.shape[:3])
    crit = np.unravel_index(np.argmax(rel[..., 10]), rel.shape[:3])
    xcc = (t[..., 6] >> 32) & 15
    spread = float(np.mean([len(set(xcc[b, h].tolist())) for b in range(B) for h in range(Hkv)]))
    print(json.dumps({"len": a.len, "batch": B, "chunk": chunk, "nsplit": nsplit, "event_us": round(us, 2),
                      "stage_us_min_p50_max": q,
                      "nonempty_stage_p50": {n: round(float(np.median(rel[..., i][nonempty])), 2)
                                             for i, n in enumerate(names)},
                      "critical_wg": {"b": int(crit[0]), "head": int(crit[1]), "split": int(crit[2]),
                                      "stages_us": [round(float(x), 2) for x in rel[crit]],
                                      "last": int(t[crit][5])},
                      "xcds_per_head": spread}), flush=True)


if __name__ == "__main__":
    main()
