"""Vector index sharded across the GPUs of a node (the vector-DB analogue of expert parallelism).

Each rank owns one in-HBM shard (flat or IVFFlat). A search is one collective round over xGMI:

    C2  all-gather of the query embeddings  [W*B, d]   (every shard scores every query)
        local fused scan + doc filter + threshold + top-k on the shard
    C1  all-gather of per-shard (score, id) top-k lists [W, W*B, k] packed into ONE int64 buffer
        (a few KB: latency-bound, so all queries of a step share ONE collective)
        device merge (topk_merge kernel) -> each rank keeps its own queries' global top-k

Exactness: the doc filter and the similarity floor are applied inside each shard BEFORE the
per-shard top-k, so the merged result equals the single-GPU exact result.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import all_gather_rows, pack_scores_ids, unpack_scores_ids
from .search_plane import merge_shard_topk


class ShardedIndex:
    def __init__(self, local, rank: int = 0, world: int = 1, group=None):
        self.local, self.rank, self.world, self.group = local, rank, world, group
        self.ops = local.ops

    def __len__(self):
        return len(self.local)

    def search(self, q_local: torch.Tensor, k: int, min_sim: float, doc_filters_all=None):
        """q_local [B, d] (same B on every rank). doc_filters_all: filters for ALL ranks' queries in
        rank order (len W*B) or None. Returns (scores fp32 [B, k], ids int64 [B, k]) on device."""
        B = q_local.shape[0]
        if self.world == 1:
            s, rows = self.local.search(q_local, k, min_sim, doc_filters_all)
            return s, self.local.gather_ids(rows)
        qs = all_gather_rows(q_local.contiguous(), self.group)                     # C2
        s, rows = self.local.search(qs, k, min_sim, doc_filters_all)
        gid = self.local.gather_ids(rows)                                          # int64 [W*B, k]
        P = all_gather_rows(pack_scores_ids(s, gid), self.group)                    # C1 (one buffer)
        S, G = unpack_scores_ids(P)
        S = S.reshape(self.world, self.world * B, k)
        G = G.reshape(self.world, self.world * B, k)
        mine = slice(self.rank * B, (self.rank + 1) * B)
        return merge_shard_topk(self.ops, S[:, mine].contiguous(), G[:, mine].contiguous(), k)

    def train(self, **kw):
        if hasattr(self.local, "train"):
            if self.world > 1:
                def allreduce(t):
                    if t.is_cuda and dist.get_backend(self.group) == "gloo":  # 1-GPU multi-rank rehearsal
                        h = t.cpu()
                        dist.all_reduce(h, group=self.group)
                        t.copy_(h)
                    else:
                        dist.all_reduce(t, group=self.group)
                self.local.allreduce = allreduce
            return self.local.train(**kw)
        return False
