"""One decode-sized GEMM shape, cold weights (a graph of calls over >= 1 GiB of weight copies), for
PMC passes and A/B of the mid-M route: python bench/midm_one.py M N K [tile] [splits] [epi]
(tile 0 = the production route; epi swiglu|plain)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from decode_gemm_sweep import timed  # noqa: E402


def main():
    M, N, Kd = (int(x) for x in sys.argv[1:4])
    tile = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    splits = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    epi = K.EPI_SWIGLU if (sys.argv[6] if len(sys.argv) > 6 else "plain") == "swiglu" else K.EPI_NONE
    x = torch.randn(M, Kd, device="cuda").bfloat16()
    by = N * Kd * 2
    ncopy = max(2, (1 << 30) // by + 1)
    ws = [(torch.randn(N, Kd, device="cuda") * 0.02).bfloat16() for _ in range(ncopy)]
    out = torch.empty(M, N // 2 if epi == K.EPI_SWIGLU else N, device="cuda", dtype=torch.bfloat16)
    K.reserve_workspace(max(1, splits) * M * N * 4 + (1 << 20), torch.device("cuda"))
    us = timed(lambda i: K.gemm(x, ws[i % ncopy], epi=epi, out=out, tile=tile, splits=splits), 2 * ncopy)
    print(f"M={M} N={N} K={Kd} tile={tile} splits={splits}: {us:.2f} us, {by / us / 1e6:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
