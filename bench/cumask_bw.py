"""HBM read bandwidth a CU subset can pull (CU-masked stream, ops/streams.py): LDS-DMA ring
(depth 8 / 16 / 31 x 1 KB per wave) vs register streaming (U = 8 / 16), 1-2 workgroups per CU.
Decides whether the HBM-bound decode attention can run on a fraction of the chip beside the
MFMA-bound prefill (profiles/r3/cumask_probe.jsonl measured the register-streaming decode kernel)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import streams as S  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L = K.lib()
    L.da_stream_probe.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    n = S.cu_count(dev)
    total = 2 << 30
    src = torch.empty(total, dtype=torch.uint8, device=dev)
    src.random_(0, 255)
    out = torch.zeros(4096, dtype=torch.int32, device=dev)
    cus_list = [int(x) for x in os.environ.get("CUS", "32,64,96,128,192,256").split(",")]
    arms = [(0, 8, 1), (0, 16, 1), (0, 31, 1), (1, 8, 1), (1, 16, 1), (1, 16, 2)]
    for cus in cus_list:
        if cus >= n:
            stream, bits = torch.cuda.Stream(device=dev), list(range(n))
        else:
            bits, _ = S.split_groups(n, cus / n)
            stream = S.masked_stream(bits, dev, tag="bw")
        res = {"cus": len(bits)}
        for mode, depth, occ in arms:
            nwg = len(bits) * occ
            per = (total // nwg) // 4096 * 4096

            def run():
                K._check(L.da_stream_probe(ctypes.c_void_p(src.data_ptr()), per, nwg, mode, depth,
                                           ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream.cuda_stream)),
                         "stream_probe")
            with torch.cuda.stream(stream):
                run()
                stream.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(3):
                    run()
                e1.record(stream)
                e1.synchronize()
            ms = e0.elapsed_time(e1) / 3
            res[f"{'lds' if mode == 0 else 'reg'}{depth}x{occ}"] = round(per * nwg / ms / 1e9, 2)  # TB/s
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
