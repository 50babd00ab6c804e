"""IVFFlat index shard: spherical k-means coarse quantizer over list-major rows in HBM.

Replaces pgvector ``ivfflat (vector vector_cosine_ops) WITH (lists = 100)`` with default
probes = 1 (internal/store/postgres.go:95-99). Unlike the reference (index
built on an empty table, Appendix B #11) centroids are trained on the stored rows:
  assign  = MFMA dense top-1 over the centroids (topk_dense, k = 1, rows as queries)
  update  = kmeans_accum (fp32 atomics) + optional cross-shard all-reduce of sums/counts (C6)
Training re-orders the row store itself into list-major order (rows, external ids and doc slots
permuted together), so there is exactly one copy of the vectors in HBM — a 288 GB part holds
~100M 1024-d bf16 rows (BASELINE config 5). ``build_streaming`` builds such an index chunk by
chunk (sample -> train -> assign pass -> scatter pass) without ever materialising an unordered
copy. Search probes the ``probes`` nearest lists per query (topk_dense over centroids) and scans
only those lists' contiguous row ranges (topk_ranges), the doc filter as a bitmap. Rows added
after training live in a delta region scanned exactly; the index retrains once the delta exceeds
``retrain_frac`` of the trained rows. Like pgvector, an IVF query may return fewer than k rows.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import h2d
from .flat import DocEntry, FlatIndex


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
        self.list_off = None    # np int64 [lists + 1]: list l = rows [list_off[l], list_off[l+1])

    # ------------------------------------------------------------------ training
    def _kmeans(self, Xs: torch.Tensor, iters: int) -> torch.Tensor:
        L = self.lists
        rng = np.random.default_rng(self.seed)
        init = torch.from_numpy(rng.choice(Xs.shape[0], size=L, replace=False)).to(self.device)
        C = Xs.index_select(0, init).float()
        if self.allreduce is not None:  # identical init across shards: average shard inits
            self.allreduce(C)
        C = torch.nn.functional.normalize(C, dim=-1)
        for _ in range(iters):
            assign = self._assign(Xs, C)
            sums = torch.zeros((L, self.dim), dtype=torch.float32, device=self.device)
            cnt = torch.zeros(L, dtype=torch.float32, device=self.device)
            self.ops.kmeans_accum(Xs, assign, sums, cnt)
            if self.allreduce is not None:
                self.allreduce(sums)
                self.allreduce(cnt)
            empty = cnt == 0
            C = torch.where(empty[:, None], C, torch.nn.functional.normalize(sums, dim=-1))
        return C.to(torch.bfloat16).contiguous()

    def train(self, iters: int = 10, sample: int | None = None):
        with self.writing():
            n = self.n
            if n < self.lists:
                return False
            X = self.X[:n]
            rng = np.random.default_rng(self.seed + 1)
            if sample is not None and sample < n:
                Xs = X.index_select(0, torch.from_numpy(rng.choice(n, sample, replace=False)).to(self.device))
            else:
                Xs = X
            self.centroids = self._kmeans(Xs.contiguous(), iters)
            self._build_lists()
            return True

    def _assign(self, rows: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
        """Nearest centroid per row. Many rows x few centroids is a GEMM (rows . C^T on the MFMA
        GEMM kernel, 64k-row slices) + row argmax; the top-k scan kernel is built for the
        opposite shape (few queries x many rows) and is only used for tiny inputs."""
        Cb = C.to(torch.bfloat16).contiguous()
        rows = rows.contiguous()
        if rows.shape[0] < 4096 or (rows.is_cuda and self.dim % 64):
            _, idx = self.ops.topk_dense(Cb, rows, 1, -2.0)
            return idx[:, 0].contiguous()
        out = torch.empty(rows.shape[0], dtype=torch.int32, device=rows.device)
        for a in range(0, rows.shape[0], 1 << 16):
            s = self.ops.gemm(rows[a:a + (1 << 16)], Cb)
            out[a:a + s.shape[0]] = torch.argmax(s, dim=1).int()
        return out

    def _assign_chunked(self, X: torch.Tensor, chunk: int = 1 << 20) -> torch.Tensor:
        out = torch.empty(X.shape[0], dtype=torch.int32, device=self.device)
        for a in range(0, X.shape[0], chunk):
            out[a:a + chunk] = self._assign(X[a:a + chunk], self.centroids)
        return out

    def _build_lists(self):
        """Permute rows, ids and slots of [0, n) into list-major order and rebuild doc ranges."""
        n = self.n
        assign = self._assign_chunked(self.X[:n])
        order = torch.sort(assign.long(), stable=True).indices
        counts = torch.bincount(assign.long(), minlength=self.lists).cpu().numpy()
        self.list_off = np.zeros(self.lists + 1, dtype=np.int64)
        np.cumsum(counts, out=self.list_off[1:])
        self.X[:n] = self.X[:n].index_select(0, order)
        self.slots_t[:n] = self.slots_t[:n].index_select(0, order)
        self.ids_t[:n] = self.ids_t[:n].index_select(0, order)
        self.ids[:n] = self.ids_t[:n].cpu().numpy()
        self._rebuild_doc_ranges(n)
        self.trained_n = n

    def _rebuild_doc_ranges(self, n: int):
        """After a list-major permutation a document's rows are scattered over the lists, so the
        IVF shard tracks documents by slot (row counts) instead of row ranges."""
        cnt = torch.bincount(self.slots_t[:n].clamp_min(0).long(), weights=(self.slots_t[:n] >= 0).float(),
                             minlength=len(self.slot_docs)).cpu().numpy() if n else np.zeros(len(self.slot_docs))
        for i, d in enumerate(self.slot_docs):
            e = self.docs[d]
            e.ranges = []
            e.rows = int(cnt[i]) if i < len(cnt) else 0

    # ------------------------------------------------------------------ bulk streaming build
    def build_streaming(self, gen_chunk, n_rows: int, chunk_rows: int, rows_per_doc: int, doc_prefix: str = "d",
                        iters: int = 10, sample: int = 1 << 20, id_base: int = 0):
        """Build a trained index of ``n_rows`` rows from ``gen_chunk(c) -> bf16 [rows, dim]`` (chunk c
        covers rows [c*chunk_rows, ...); must be deterministic: it is called twice per chunk).
        Documents are ``rows_per_doc`` consecutive generated rows named f"{doc_prefix}{i}"; external
        ids are id_base + generation index. Peak memory = the final index + one chunk."""
        with self.writing():
            if self.n:
                raise RuntimeError("build_streaming needs an empty index")
            nch = (n_rows + chunk_rows - 1) // chunk_rows
            # 1) train on a sample drawn evenly from the chunks
            per = max(self.lists, sample // nch)
            parts = []
            for c in range(nch):
                x = gen_chunk(c)
                parts.append(x[torch.randperm(x.shape[0], device=self.device)[:per]].clone())
                del x
            Xs = torch.cat(parts)[:max(sample, self.lists)].contiguous()
            del parts
            self.centroids = self._kmeans(Xs, iters)
            del Xs
            # 2) assignment pass -> list sizes
            assign = torch.empty(n_rows, dtype=torch.int32, device=self.device)
            for c in range(nch):
                a = c * chunk_rows
                x = gen_chunk(c)
                assign[a:a + x.shape[0]] = self._assign_chunked(x)
                del x
            counts = torch.bincount(assign.long(), minlength=self.lists)
            off_t = torch.zeros(self.lists + 1, dtype=torch.int64, device=self.device)
            off_t[1:] = torch.cumsum(counts, 0)
            # destination of every generated row: list offset + rank within its list (stable)
            order = torch.sort(assign.long(), stable=True).indices
            dest = torch.empty(n_rows, dtype=torch.int64, device=self.device)
            dest[order] = torch.arange(n_rows, device=self.device)
            del order, assign
            # 3) scatter pass into an exactly-sized list-major store
            self.X = torch.empty((n_rows, self.dim), dtype=torch.bfloat16, device=self.device)
            gen_idx = torch.arange(n_rows, device=self.device)
            self.slots_t = torch.empty(n_rows, dtype=torch.int32, device=self.device)
            self.slots_t[dest] = (gen_idx // rows_per_doc).int()
            self.ids_t = torch.empty(n_rows, dtype=torch.int64, device=self.device)
            self.ids_t[dest] = gen_idx + id_base
            del gen_idx
            for c in range(nch):
                a = c * chunk_rows
                x = gen_chunk(c)
                self.X[dest[a:a + x.shape[0]]] = x
                del x
            del dest
            self.ids = self.ids_t.cpu().numpy()
            ndocs = (n_rows + rows_per_doc - 1) // rows_per_doc
            self.slot_docs = [f"{doc_prefix}{i}" for i in range(ndocs)]
            self.docs = {d: DocEntry(slot=i) for i, d in enumerate(self.slot_docs)}
            self.n = n_rows
            self.list_off = off_t.cpu().numpy()
            self._rebuild_doc_ranges(n_rows)
            self.trained_n = n_rows
            return self

    def add(self, doc_id: str, ids: np.ndarray, vecs: torch.Tensor) -> tuple[int, int]:
        r = super().add(doc_id, ids, vecs)  # delta region: contiguous ranges kept until retraining
        return r

    def remove_doc(self, doc_id: str) -> int:
        with self.writing():
            e = self.docs.get(doc_id)
            if e is None or e.rows == 0:
                return 0
            s = self.slots_t[:self.n]
            s.masked_fill_(s == e.slot, -1)
            n = e.rows
            e.ranges, e.rows = [], 0
            return n

    def live_rows_by_doc(self):
        """(rows grouped by document, [(doc_id, n_rows)]) for snapshots."""
        with self.reading():
            return self._live_rows_by_doc()

    def _live_rows_by_doc(self):
        n = self.n
        s = self.slots_t[:n].long()
        live = torch.nonzero(s >= 0).flatten()
        order = live[torch.sort(s[live], stable=True).indices]
        cnt = torch.bincount(s[live], minlength=len(self.slot_docs)).cpu().numpy()
        docs = [(d, int(cnt[i])) for i, d in enumerate(self.slot_docs) if cnt[i] > 0]
        return order.cpu().numpy(), docs

    # ------------------------------------------------------------------ search
    def search(self, q: torch.Tensor, k: int, min_sim: float, doc_filters=None):
        with self.reading():
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
            if probes <= 32:
                _, lists = self.ops.topk_dense(self.centroids, q, probes, -2.0)
            else:  # wide probing: centroid scores as one GEMM, then torch top-k
                lists = torch.topk(self.ops.gemm(q, self.centroids).float(), probes, dim=1).indices.int()
            lists_h = lists.cpu().numpy()
            off = self.list_off
            starts, ends = off[lists_h.clip(0)], off[lists_h.clip(0) + 1]
            valid = (lists_h >= 0) & (ends > starts)
            per_q = np.where(valid, ends - starts, 0).sum(axis=1)
            maxrows = int(per_q.max()) if Q else 0
            bitmap = None if doc_filters is None else self._bitmap(Q, doc_filters)
            if maxrows > 0:
                rr = np.stack([starts[valid], ends[valid]], axis=1).astype(np.int32)
                ro = np.zeros(Q + 1, dtype=np.int32)
                np.cumsum(valid.sum(axis=1), out=ro[1:])
                rt = h2d(rr, self.device)
                ot = h2d(ro, self.device)
                s1, i1 = self.ops.topk_ranges(self.X, q, rt, ot, k, min_sim, max_rows=maxrows,
                                              slots=self.slots_t, bitmap=bitmap)
            else:
                s1 = torch.full((Q, k), float("-inf"), device=self.device)
                i1 = torch.full((Q, k), -1, dtype=torch.int32, device=self.device)
            if self.n > self.trained_n:  # delta rows: exact scan
                d0 = self.trained_n
                rt = h2d(np.asarray([[d0, self.n]] * Q, dtype=np.int32), self.device)
                ot = torch.arange(Q + 1, dtype=torch.int32, device=self.device)
                s2, i2 = self.ops.topk_ranges(self.X, q, rt, ot, k, min_sim, max_rows=self.n - d0,
                                              slots=self.slots_t, bitmap=bitmap)
                s1, i1 = self.ops.topk_merge(torch.stack([s1, s2]), torch.stack([i1, i2]), k)
            return s1, i1

    def _bitmap(self, Q, doc_filters):
        nslots = len(self.slot_docs)
        W = (nslots + 1 + 31) // 32
        bm = np.zeros((Q, W), dtype=np.uint32)
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
        return h2d(bm.view(np.int32), self.device)
