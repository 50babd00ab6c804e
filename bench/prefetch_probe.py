"""Probe: does reading the NEXT decode GEMM's weights on a side stream (MALL prefetch) speed up a
latency-bound chain of decode GEMMs? Phi-3-mini layer shapes x 32 layers (7.2 GB of weights, far
larger than the 256 MB Infinity Cache), captured in one HIP graph, replayed; M = decode batch."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--out", default="")
    ap.add_argument("--blas", action="store_true")
    ap.add_argument("--swiglu", action="store_true", help="gate/up with the SwiGLU epilogue (fused vs separate)")
    ap.add_argument("--ms", default="1,8,16,32,64,128")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H, I = 3072, 8192
    shapes = [(3 * H, H), (H, H), (2 * I, H), (H, I)]
    g = torch.Generator(device=dev).manual_seed(0)
    W = [[(torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16) for n, k in shapes]
         for _ in range(a.layers)]
    gb = sum(w.numel() * 2 for L in W for w in L) / 1e9

    if a.blas:  # same chain, hipBLASLt (torch.matmul) vs the in-tree decode GEMM tiles
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, I, device=dev).to(torch.bfloat16)
            outs = [torch.empty(M, n, device=dev, dtype=torch.bfloat16) for n, _ in shapes]
            act = torch.empty(M, I, device=dev, dtype=torch.bfloat16)  # SwiGLU output of gate/up
            for impl in ("da", "blas"):
                def run():
                    for L in W:
                        for j, w in enumerate(L):
                            xi = x[:, :w.shape[1]]
                            if impl == "da":
                                if j == 2 and a.swiglu:
                                    K.gemm(xi, w, epi=K.EPI_SWIGLU, out=act)
                                else:
                                    K.gemm(xi, w, out=outs[j])
                            else:
                                torch.matmul(xi, w.t(), out=outs[j])
                                if j == 2 and a.swiglu:
                                    K.swiglu_interleaved(outs[j], act)
                run(); torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    run()
                graph.replay(); torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    graph.replay()
                e.record(); torch.cuda.synchronize()
                ms = s.elapsed_time(e) / 10
                print(json.dumps({"probe": "chain_impl", "M": M, "impl": impl, "ms": round(ms, 3),
                                  "TBps": round(gb / ms, 2)}), flush=True)
                del graph
        return

    # standalone prefetch bandwidth (sanity check of the kernel)
    flat = [w for L in W for w in L]
    for nwg in (256, 1024, 4096):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for w in flat:
            K.mall_prefetch(w, nwg)
        e.record(); torch.cuda.synchronize()
        print(json.dumps({"probe": "prefetch_bw", "nwg": nwg, "TBps": round(gb / s.elapsed_time(e), 2)}), flush=True)

    res = []
    for M in (1, 16, 64):
        x = torch.randn(M, I, device=dev).to(torch.bfloat16)
        outs = [torch.empty(M, n, device=dev, dtype=torch.bfloat16) for n, _ in shapes]
        ops = []
        for L in W:
            for j, w in enumerate(L):
                ops.append((w, x[:, :w.shape[1]], outs[j]))
        for nwg, ahead in ((0, 0), (16, 1), (32, 1), (64, 1), (128, 1), (32, 2)):
            side = torch.cuda.Stream()
            graph = torch.cuda.CUDAGraph()
            K.gemm(ops[0][1], ops[0][0], out=ops[0][2])  # warm any lazy init outside capture
            torch.cuda.synchronize()
            with torch.cuda.graph(graph):
                main_s = torch.cuda.current_stream()
                for i, (w, xi, o) in enumerate(ops):
                    if nwg and i + ahead < len(ops):
                        ev = torch.cuda.Event()
                        ev.record(main_s)
                        side.wait_event(ev)
                        with torch.cuda.stream(side):
                            K.mall_prefetch(ops[i + ahead][0], nwg)
                    K.gemm(xi, w, out=o)
                if nwg:
                    main_s.wait_stream(side)
            graph.replay(); torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            s.record()
            for _ in range(reps):
                graph.replay()
            e.record(); torch.cuda.synchronize()
            ms = s.elapsed_time(e) / reps
            r = {"probe": "chain", "M": M, "nwg": nwg, "ahead": ahead, "ms": round(ms, 3),
                 "TBps": round(gb / ms, 2)}
            print(json.dumps(r), flush=True)
            res.append(r)
            del graph
    if a.out:
        with open(a.out, "w") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
