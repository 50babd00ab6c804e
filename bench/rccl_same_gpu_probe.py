"""Probe: can two ranks use RCCL on ONE GPU (to rehearse the nccl-only paths on a 1-GPU box)?
torchrun --nproc-per-node 2 bench/rccl_same_gpu_probe.py  -> one JSON line from rank 0."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    out = {"rank": r, "world": w}
    t0 = time.time()
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.ones(1024, device="cuda") * (r + 1)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["all_reduce"] = float(x[0])
        # a collective captured in a HIP graph (the served TP fallback form)
        s = torch.cuda.Stream()
        y = torch.ones(1024, device="cuda")
        with torch.cuda.stream(s):
            for _ in range(2):
                dist.all_reduce(y)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        y.fill_(r + 1)
        with torch.cuda.graph(g):
            dist.all_reduce(y)
        y.fill_(r + 1)
        g.replay()
        torch.cuda.synchronize()
        out["graph_all_reduce"] = float(y[0])
        out["ok"] = True
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)[:500]
    out["s"] = round(time.time() - t0, 2)
    if r == 0:
        print(json.dumps(out), flush=True)
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
