"""Flash prefill dispatch order A/B (attention.hip fa_block, da_set_flash_rev): grid order with
causal longest-first (rev 1) vs the same plus XCD-grouped (sequence, kv head) pairs (rev 3), on the
default kernel of each shape. Interleaved rounds, best of ROUNDS; outputs must be bit-identical
(the order changes nothing but where and when a block runs). One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    rounds = int(os.environ.get("ROUNDS", "3"))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = [("phi3_qa_chunk", 22, 2938, 32, 32, 96, True), ("phi3_b8", 8, 2944, 32, 32, 96, True),
              ("phi3_b1", 1, 2888, 32, 32, 96, True), ("bge_base", 64, 512, 12, 12, 64, False),
              ("llama3_prefill", 4, 4096, 32, 8, 128, True)]
    for name, B, L, H, Hkv, D, causal in shapes:
        T = B * L
        qkv = torch.randn(T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
        cu = torch.arange(0, T + 1, L, device=dev, dtype=torch.int32)
        fl = 4 * B * L * L * H * D * (0.5 if causal else 1.0)
        best, outs = {}, {}
        for _ in range(rounds):
            for rev in (1, 3):
                K.lib().da_set_flash_rev(rev)
                t = timeit(lambda: K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal))
                best[rev] = min(best.get(rev, 1e9), t)
                outs[rev] = K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal)
        K.lib().da_set_flash_rev(3)
        torch.cuda.synchronize()
        print(json.dumps({"shape": name, "B": B, "L": L, "ms": {f"rev{r}": round(t, 3) for r, t in best.items()},
                          "tflops": {f"rev{r}": round(fl / t / 1e9, 1) for r, t in best.items()},
                          "identical": bool(torch.equal(outs[1], outs[3]))}), flush=True)


if __name__ == "__main__":
    main()
