"""BASELINE config 4's index at its real total size: recall of the sharded search vs ONE exact index.

Every rank builds the bench's synthetic shard (bench.shard_vectors / bench.doc_names, e.g. 8 x 1.25M
rows = the 10M-chunk index sharded 8-way) and runs ``ShardedIndex.search`` (C2 all-gather of the
query rows, fused scan + filter + top-k per shard, C1 all-gather of the per-shard top-k, device
merge) on its B queries, unfiltered (the global top-k over all rows) and filtered the way bench.py's
QA step filters (docs_per_query documents on random shards). Rank 0 then regenerates every shard
from its seed, scores ALL W x B queries against the whole index in fp32 (torch, shard by shard) and
reports recall@k of the sharded answer against that exact answer. The reference's search is
``Store.TopK`` (internal/store/postgres.go:218-285): one exact query over one table.

  python -m torch.distributed.run --nproc-per-node 8 bench/sharded_recall.py --rows 1250000 --dim 1024
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import doc_names, shard_vectors  # noqa: E402
from docagents_amd.index import make_index  # noqa: E402
from docagents_amd.parallel.dist import init_from_env  # noqa: E402
from docagents_amd.parallel.sharded_index import ShardedIndex  # noqa: E402


def exact(Qall: torch.Tensor, W: int, rows: int, d: int, k: int, dev, masks=None):
    """fp32 exact top-k of every query over the W regenerated shards. masks: per query a list of
    (shard, row0, row1) ranges it may see (None = all rows)."""
    best_s = torch.full((Qall.shape[0], 0), float("-inf"), device=dev)
    best_i = torch.zeros((Qall.shape[0], 0), dtype=torch.int64, device=dev)
    q = Qall.float()
    for r in range(W):
        X = shard_vectors(r, rows, d, dev)
        gid = np.int64(r) * 1_000_000_000 + torch.arange(rows, device=dev, dtype=torch.int64)
        for c0 in range(0, rows, 1 << 18):
            Xc = X[c0:c0 + (1 << 18)].float()
            s = q @ Xc.T
            if masks is not None:
                m = torch.zeros_like(s, dtype=torch.bool)
                for qi, rng in enumerate(masks):
                    for (sr, a, b) in rng:
                        if sr == r:
                            a2, b2 = max(a, c0), min(b, c0 + Xc.shape[0])
                            if a2 < b2:
                                m[qi, a2 - c0:b2 - c0] = True
                s = s.masked_fill(~m, float("-inf"))
            kk = min(k, s.shape[1])
            ts, ti = s.topk(kk, dim=1)
            best_s = torch.cat([best_s, ts], 1)
            best_i = torch.cat([best_i, gid[c0:c0 + Xc.shape[0]][ti]], 1)
            o = best_s.topk(min(k, best_s.shape[1]), dim=1)
            best_s, best_i = o.values, best_i.gather(1, o.indices)
        del X
    best_i = torch.where(torch.isinf(best_s), torch.full_like(best_i, -1), best_i)
    return best_s, best_i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_250_000, help="rows per shard")
    ap.add_argument("--dim", type=int, default=1024, help="1024 = BGE-large")
    ap.add_argument("--queries", type=int, default=64, help="total over the world")
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--chunks-per-doc", type=int, default=10)
    ap.add_argument("--docs-per-query", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    info = init_from_env()
    W, R, dev = info.world, info.rank, info.device
    B = a.queries // W
    t0 = time.perf_counter()
    idx = make_index("flat", a.dim, dev)
    ndocs = a.rows // a.chunks_per_doc
    names = doc_names(W, ndocs)
    X = shard_vectors(R, a.rows, a.dim, dev)
    idx.add_bulk(names[R], [a.chunks_per_doc] * ndocs, np.int64(R) * 1_000_000_000 + np.arange(a.rows, dtype=np.int64), X)
    del X
    shard = ShardedIndex(idx, R, W)
    t_build = time.perf_counter() - t0
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    Qall = torch.nn.functional.normalize(torch.randn((B * W, a.dim), device=dev, generator=g), dim=-1).to(torch.bfloat16)
    mine = Qall[R * B:(R + 1) * B].contiguous()
    rng = np.random.default_rng(5)
    fl = [[(int(r), int(j)) for r, j in zip(rng.integers(0, W, a.docs_per_query), rng.integers(0, ndocs, a.docs_per_query))]
          for _ in range(B * W)]
    filters_all = [[names[r][j] for r, j in f] for f in fl]
    res = {}
    for mode, flt in (("unfiltered", None), ("filtered", filters_all)):
        dist.barrier() if W > 1 else None
        t1 = time.perf_counter()
        s, ids = shard.search(mine, a.k, -1.0, flt)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t1
        got = [None] * W
        if W > 1:
            dist.all_gather_object(got, ids.cpu().numpy())
        else:
            got = [ids.cpu().numpy()]
        res[mode] = (np.concatenate(got, 0), dt)
    out = None
    if R == 0:
        out = {"world": W, "rows_per_shard": a.rows, "rows_total": W * a.rows, "dim": a.dim, "queries": B * W,
               "k": a.k, "backend": info.backend, "build_s": round(t_build, 1)}
        for mode, (ids, dt) in res.items():
            masks = None
            if mode == "filtered":
                masks = [[(r, j * a.chunks_per_doc, (j + 1) * a.chunks_per_doc) for r, j in f] for f in fl]
            t2 = time.perf_counter()
            _, ref = exact(Qall, W, a.rows, a.dim, a.k, dev, masks)
            ref = ref.cpu().numpy()
            hit = sum(len(set(ids[q][ids[q] >= 0]) & set(ref[q][ref[q] >= 0])) for q in range(len(ref)))
            want = int((ref >= 0).sum())
            out[mode] = {"recall_at_k": round(hit / max(1, want), 6), "hits": hit, "expected": want,
                         "rows_identical": int(sum(np.array_equal(ids[q], ref[q]) for q in range(len(ref)))),
                         "sharded_search_ms": round(dt * 1000, 2), "exact_s": round(time.perf_counter() - t2, 1)}
        print(json.dumps(out), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    if W > 1:
        dist.barrier()
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
