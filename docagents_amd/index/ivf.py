"""IVFFlat index shard: spherical k-means coarse quantizer + list-major packed rows.

Replaces pgvector ``ivfflat (vector vector_cosine_ops) WITH (lists = 100)`` with default
probes = 1 (internal/store/postgres.go:95-99). Unlike the reference (index
built on an empty table, Appendix B #11) centroids are trained on the stored rows:
  assign  = MFMA dense top-1 over the centroids (topk_dense, k = 1, rows as queries)
  update  = kmeans_accum (fp32 atomics) + optional cross-shard all-reduce of sums/counts (C6)
Search probes the ``probes`` nearest lists per query (topk_dense over centroids) and scans only
those lists' contiguous row ranges with the doc filter as a bitmap (topk_ranges). Rows added after
training live in a delta region scanned exactly; the index retrains once the delta exceeds
``retrain_frac`` of the trained rows. Like pgvector, an IVF query may return fewer than k rows.
"""
from __future__ import annotations

import numpy as np
import torch

from .flat import FlatIndex


class IVFFlatIndex(FlatIndex):
    kind = "ivfflat"

    def __init__(self, dim: int, device="cuda", lists: int = 100, probes: int = 1, capacity: int = 1024,
                 retrain_frac: float = 0.25, allreduce=None, seed: int = 0):
        super().__init__(dim, device, capacity)
        self.lists, self.probes = lists, probes
        self.retrain_frac = retrain_frac
        self.allreduce = allreduce  # callable(tensor) -> None, sums in place across shards
        self.seed = seed
        self.centroids = None
        self.trained_n = 0
        self.Xp = None          # list-major copy of the trained rows
        self.perm = None        # int64 np: list-major position -> row
        self.slots_p = None
        self.list_off = None    # np int64 [lists + 1]

    # ------------------------------------------------------------------ training
    def train(self, iters: int = 10, sample: int | None = None):
        with self.lock:
            n = self.n
            L = self.lists
            if n < L:
                return False
            X = self.X[:n]
            rng = np.random.default_rng(self.seed)
            init = torch.from_numpy(rng.choice(n, size=L, replace=False)).to(self.device)
            C = X.index_select(0, init).float()
            if self.allreduce is not None:  # identical init across shards: average shard inits
                self.allreduce(C)
            C = torch.nn.functional.normalize(C, dim=-1)
            Xs = X if sample is None or sample >= n else X[torch.from_numpy(rng.choice(n, sample, replace=False)).to(self.device)]
            for _ in range(iters):
                assign = self._assign(Xs, C)
                sums = torch.zeros((L, self.dim), dtype=torch.float32, device=self.device)
                cnt = torch.zeros(L, dtype=torch.float32, device=self.device)
                self.ops.kmeans_accum(Xs, assign, sums, cnt)
                if self.allreduce is not None:
                    self.allreduce(sums)
                    self.allreduce(cnt)
                empty = cnt == 0
                newC = torch.nn.functional.normalize(sums, dim=-1)
                C = torch.where(empty[:, None], C, newC)
            self.centroids = C.to(torch.bfloat16).contiguous()
            self._build_lists()
            return True

    def _assign(self, rows: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
        Cb = C.to(torch.bfloat16).contiguous()
        _, idx = self.ops.topk_dense(Cb, rows.contiguous(), 1, -2.0)
        return idx[:, 0].contiguous()

    def _build_lists(self):
        n = self.n
        assign = self._assign(self.X[:n], self.centroids).cpu().numpy().astype(np.int64)
        order = np.argsort(assign, kind="stable")
        counts = np.bincount(assign, minlength=self.lists)
        self.list_off = np.zeros(self.lists + 1, dtype=np.int64)
        np.cumsum(counts, out=self.list_off[1:])
        self.perm = order
        pt = torch.from_numpy(order).to(self.device)
        self.Xp = self.X[:n].index_select(0, pt).contiguous()
        self.slots_p = self.slots_t[:n].index_select(0, pt).contiguous()
        self.trained_n = n

    def remove_doc(self, doc_id: str) -> int:
        r = super().remove_doc(doc_id)
        if self.slots_p is not None and r:
            # refresh the list-major slot copy so removed rows stop matching
            pt = torch.from_numpy(self.perm).to(self.device)
            self.slots_p = self.slots_t[:self.trained_n].index_select(0, pt).contiguous()
        return r

    # ------------------------------------------------------------------ search
    def search(self, q: torch.Tensor, k: int, min_sim: float, doc_filters=None):
        with self.lock:
            if self.centroids is None or self.n < self.lists:
                if self.n >= self.lists and self.n >= 4 * self.lists:
                    self.train()
                if self.centroids is None:
                    return super().search(q, k, min_sim, doc_filters)
            if self.n - self.trained_n > self.retrain_frac * max(1, self.trained_n):
                self.train()
            Q = q.shape[0]
            q = q.to(device=self.device, dtype=torch.bfloat16).contiguous()
            probes = min(self.probes, self.lists)
            _, lists = self.ops.topk_dense(self.centroids, q, probes, -2.0)
            lists_h = lists.cpu().numpy()
            ranges, off, maxrows = [], [0], 0
            for i in range(Q):
                tot = 0
                for l in lists_h[i]:
                    if l < 0:
                        continue
                    a, b = int(self.list_off[l]), int(self.list_off[l + 1])
                    if b > a:
                        ranges.append((a, b))
                        tot += b - a
                off.append(len(ranges))
                maxrows = max(maxrows, tot)
            bitmap = self._bitmap(Q, doc_filters)
            if maxrows > 0:
                rt = torch.tensor(ranges, dtype=torch.int32, device=self.device).view(-1, 2)
                ot = torch.tensor(off, dtype=torch.int32, device=self.device)
                s1, i1 = self.ops.topk_ranges(self.Xp, q, rt, ot, k, min_sim, max_rows=maxrows,
                                              slots=self.slots_p, bitmap=bitmap)
                permt = torch.from_numpy(self.perm).to(self.device)
                i1 = torch.where(i1 >= 0, permt[i1.clamp_min(0).long()].int(), i1)
            else:
                s1 = torch.full((Q, k), float("-inf"), device=self.device)
                i1 = torch.full((Q, k), -1, dtype=torch.int32, device=self.device)
            if self.n > self.trained_n:  # delta rows: exact scan
                d0 = self.trained_n
                Xd = self.X[d0:self.n]
                rt = torch.tensor([[0, self.n - d0]] * Q, dtype=torch.int32, device=self.device)
                ot = torch.arange(Q + 1, dtype=torch.int32, device=self.device)
                s2, i2 = self.ops.topk_ranges(Xd.contiguous(), q, rt, ot, k, min_sim, max_rows=self.n - d0,
                                              slots=self.slots_t[d0:self.n].contiguous(), bitmap=bitmap)
                i2 = torch.where(i2 >= 0, i2 + d0, i2)
                s1, i1 = self.ops.topk_merge(torch.stack([s1, s2]), torch.stack([i1, i2]), k)
            return s1, i1

    def _bitmap(self, Q, doc_filters):
        nslots = len(self.slot_docs)
        W = (nslots + 1 + 31) // 32
        bm = np.zeros((Q, W), dtype=np.uint32)
        if doc_filters is None:
            full, rem = divmod(nslots, 32)
            bm[:, :full] = 0xFFFFFFFF
            if rem:
                bm[:, full] = (1 << rem) - 1
        else:
            full, rem = divmod(nslots, 32)
            for i, f in enumerate(doc_filters):
                if f is None:
                    bm[i, :full] = 0xFFFFFFFF
                    if rem:
                        bm[i, full] = (1 << rem) - 1
                    continue
                for d in f:
                    e = self.docs.get(d)
                    if e is not None and e.rows:
                        bm[i, e.slot >> 5] |= np.uint32(1 << (e.slot & 31))
        return torch.from_numpy(bm.view(np.int32)).to(self.device)
