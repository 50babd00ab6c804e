"""Vector-index benchmark on one MI355X (BASELINE configs 4 and 5: 10M-chunk flat shard,
100M-chunk IVFFlat in HBM). Synthetic clustered unit vectors (topic centres + noise, generated
deterministically chunk by chunk on the GPU); reports build time, HBM footprint, batch search
latency / QPS with and without a document filter, and IVF recall@k against the exact scan.

  python bench/index_bench.py --kind flat --rows 10000000 --dim 1024
  python bench/index_bench.py --kind ivfflat --rows 100000000 --dim 1024 --lists 8192 --probes 8,32
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.index.flat import FlatIndex  # noqa: E402
from docagents_amd.index.ivf import IVFFlatIndex  # noqa: E402


def make_gen(dim: int, chunk: int, n_rows: int, centres: int = 65536, sigma: float = 0.35, seed: int = 0):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    C = torch.nn.functional.normalize(torch.randn(centres, dim, device=dev, generator=g), dim=-1)

    def gen(c: int) -> torch.Tensor:
        rows = min(chunk, n_rows - c * chunk)
        gg = torch.Generator(device=dev)
        gg.manual_seed(seed * 1_000_003 + c + 1)
        lab = torch.randint(0, centres, (rows,), device=dev, generator=gg)
        x = C[lab] + sigma / dim ** 0.5 * torch.randn(rows, dim, device=dev, generator=gg)
        return torch.nn.functional.normalize(x, dim=-1).to(torch.bfloat16)
    return gen, C


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="flat", choices=("flat", "ivfflat"))
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=1 << 21)
    ap.add_argument("--rows-per-doc", type=int, default=1000)
    ap.add_argument("--lists", type=int, default=8192)
    ap.add_argument("--probes", default="8,32")
    ap.add_argument("--batches", default="1,64,512")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    gen, C = make_gen(a.dim, a.chunk, a.rows)
    nch = (a.rows + a.chunk - 1) // a.chunk
    res = {"kind": a.kind, "rows": a.rows, "dim": a.dim, "k": a.k}
    t0 = time.perf_counter()
    if a.kind == "flat":
        ix = FlatIndex(a.dim, dev, capacity=a.rows)
        ndoc = (a.rows + a.rows_per_doc - 1) // a.rows_per_doc
        for c in range(nch):
            x = gen(c)
            r0 = c * a.chunk
            d0, d1 = r0 // a.rows_per_doc, (r0 + x.shape[0] - 1) // a.rows_per_doc
            per = [min((d + 1) * a.rows_per_doc, r0 + x.shape[0]) - max(d * a.rows_per_doc, r0) for d in range(d0, d1 + 1)]
            # documents that straddle chunks get two entries under the same id (ranges append)
            ix.add_bulk([f"d{d}" for d in range(d0, d1 + 1)], per, np.arange(r0, r0 + x.shape[0]), x)
        del ndoc
    else:
        ix = IVFFlatIndex(a.dim, dev, lists=a.lists, probes=1).build_streaming(
            gen, a.rows, a.chunk, a.rows_per_doc, iters=8, sample=min(a.rows, 64 * a.lists))
    torch.cuda.synchronize()
    res["build_s"] = round(time.perf_counter() - t0, 2)
    res["hbm_index_gb"] = round(ix.X.numel() * 2 / 1e9, 2)
    res["hbm_allocated_gb"] = round(torch.cuda.memory_allocated() / 1e9, 2)
    print(json.dumps(res), flush=True)

    gq = torch.Generator(device=dev)
    gq.manual_seed(4242)
    probes = [int(p) for p in a.probes.split(",")] if a.kind == "ivfflat" else [0]
    for B in [int(b) for b in a.batches.split(",")]:
        lab = torch.randint(0, C.shape[0], (B,), device=dev, generator=gq)
        q = torch.nn.functional.normalize(C[lab] + 0.35 / a.dim ** 0.5 * torch.randn(B, a.dim, device=dev, generator=gq),
                                          dim=-1).to(torch.bfloat16)
        # exact reference over the whole store
        es, ei = ix.ops.topk_dense(ix.X[:ix.n].contiguous(), q, a.k, -2.0)
        exact_ids = ix.gather_ids(ei).cpu().numpy()
        t_exact = timeit(lambda: ix.ops.topk_dense(ix.X[:ix.n].contiguous(), q, a.k, -2.0), reps=3)
        entry = {"batch": B, "exact_scan_ms": round(t_exact * 1e3, 3),
                 "exact_scan_tbps": round(ix.n * a.dim * 2 / t_exact / 1e12, 2)}
        filt = [[f"d{(i * 7919) % max(1, a.rows // a.rows_per_doc)}" for i in range(b, b + 8)] for b in range(B)]
        for p in probes:
            if a.kind == "ivfflat":
                ix.probes = p
            t = timeit(lambda: ix.search(q, a.k, -1.0, None))
            s, r = ix.search(q, a.k, -1.0, None)
            got = ix.gather_ids(r).cpu().numpy()
            rec = float(np.mean([len(set(exact_ids[i]) & set(got[i])) / a.k for i in range(B)]))
            tf = timeit(lambda: ix.search(q, a.k, -1.0, filt), reps=3)
            key = f"probes{p}" if a.kind == "ivfflat" else "search"
            entry[key] = {"ms": round(t * 1e3, 3), "qps": round(B / t, 1), f"recall@{a.k}": round(rec, 4),
                          "filtered_8docs_ms": round(tf * 1e3, 3)}
        res[f"B{B}"] = entry
        print(json.dumps(entry), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
