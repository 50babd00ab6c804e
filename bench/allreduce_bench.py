"""All-reduce latency: xGMI IPC kernel (one-shot / two-shot) vs RCCL, per message size.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench/allreduce_bench.py

On a multi-GPU node (one rank per GPU) both paths are timed. With more ranks than GPUs (the 1-GPU
rehearsal: DA_DIST_BACKEND=gloo, ranks share the card) only the IPC kernel is timed — RCCL refuses
two ranks on one device — and the numbers are the kernel's own overhead (flag round trips and
staging), not xGMI transfer time. Each size: 20 warm-up calls, then the mean of 200 calls
captured in one HIP graph (what a decode step replays), plus the eager per-call time.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from docagents_amd.parallel.dist import init_from_env  # noqa: E402
from docagents_amd.parallel.xgmi_allreduce import XgmiAllReduce  # noqa: E402


def main():
    info = init_from_env()
    dev = info.device
    W = info.world
    shared = torch.cuda.device_count() < W
    ar = XgmiAllReduce(None, dev, max_bytes=32 << 20)
    sizes = [16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]
    rows = []
    for nb in sizes:
        t = torch.randn(nb // 2, device=dev).to(torch.bfloat16)
        res = {"bytes": nb, "path": "oneshot" if nb <= ar.oneshot_max else "twoshot"}
        for _ in range(20):
            ar.all_reduce_(t)
        torch.cuda.synchronize()
        dist.barrier()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            ar.all_reduce_(t)
        torch.cuda.synchronize()
        res["xgmi_eager_us"] = round((time.perf_counter() - t0) / n * 1e6, 2)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(50):
                ar.all_reduce_(t)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
        res["xgmi_graph_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
        if not shared and dist.get_backend() == "nccl":
            for _ in range(20):
                dist.all_reduce(t)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                dist.all_reduce(t)
            torch.cuda.synchronize()
            res["rccl_eager_us"] = round((time.perf_counter() - t0) / n * 1e6, 2)
        rows.append(res)
    ar.check()
    if info.rank == 0:
        print(json.dumps({"world": W, "ranks_share_gpu": shared, "results": rows}), flush=True)
    ar.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
