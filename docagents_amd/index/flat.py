"""In-HBM flat (brute-force) vector index shard.

Replaces the pgvector ``embeddings`` table + cosine search (internal/store/postgres.go:84,176-201,
218-285). Rows are unit-norm bf16 vectors stored contiguously in HBM; all rows
of one document are appended together, so a document filter becomes a list of row ranges and a
filtered query reads only the rows it can match (exact, filter-before-top-k semantics — pgvector
post-filters). Unfiltered / wide queries run the MFMA dense scan with a doc bitmap.

Capacity grows geometrically; at 288 GB per GPU a 768-d bf16 shard holds ~180M rows.
"""
from __future__ import annotations

import contextlib
import math
import threading
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import get_ops, h2d


@dataclass
class DocEntry:
    slot: int
    ranges: list = field(default_factory=list)  # [(start, end)]
    rows: int = 0


class FlatIndex:
    kind = "flat"

    def __init__(self, dim: int, device="cuda", capacity: int = 1024, dtype=torch.bfloat16):
        self.dim = dim
        self.device = torch.device(device)
        self.ops = get_ops(self.device)
        self.X = torch.zeros((max(64, capacity), dim), dtype=dtype, device=self.device)
        self.slots_t = torch.full((self.X.shape[0],), -1, dtype=torch.int32, device=self.device)
        self.n = 0
        self.ids = np.zeros(self.X.shape[0], dtype=np.int64)     # external chunk id per row
        self.ids_t = torch.zeros(self.X.shape[0], dtype=torch.int64, device=self.device)  # device mirror
        self.docs: dict[str, DocEntry] = {}
        self.slot_docs: list[str | None] = []
        self.lock = threading.RLock()
        self._write_ev = None   # event after the last mutation's device work (None: nothing pending)
        self._read_evs: dict = {}  # reader stream handle -> event after its last read
        self._depth = 0

    # ----------------------------------------------------------------- stream ordering
    # Writers (add / add_bulk / remove_* / _grow / IVF train) and readers (search, gather_ids,
    # snapshots) run on different HIP streams: the engine's GPU thread mutates, the search plane's
    # stream scans. Host state (n, ranges, docs) changes under ``lock`` at once, the device copies
    # later in stream order, so a reader that only took the lock could scan rows whose copy (or
    # _grow zero-fill) has not run yet. Inside the lock every mutation therefore orders its stream
    # after the previous write and every read still in flight, and records a write event as its
    # last step; every read orders its stream after that event and records a read event for its
    # stream. All device-side: no host synchronisation on either path. A committed mutation is
    # atomic to readers, as a committed INSERT is in the reference (internal/store/postgres.go:176-201).
    @contextlib.contextmanager
    def writing(self):
        with self.lock:
            cuda = self.device.type == "cuda"
            outer = self._depth == 0
            self._depth += 1
            if cuda and outer:
                st = torch.cuda.current_stream(self.device)
                if self._write_ev is not None:
                    st.wait_event(self._write_ev)
                for ev in self._read_evs.values():
                    st.wait_event(ev)
            try:
                yield
            finally:
                self._depth -= 1
                if cuda and outer:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.device))
                    self._write_ev = ev
                    self._read_evs.clear()  # this write is ordered after every one of them

    @contextlib.contextmanager
    def reading(self):
        with self.lock:
            cuda = self.device.type == "cuda"
            if cuda and self._write_ev is not None:
                torch.cuda.current_stream(self.device).wait_event(self._write_ev)
            try:
                yield
            finally:
                if cuda:
                    st = torch.cuda.current_stream(self.device)
                    ev = torch.cuda.Event()
                    ev.record(st)
                    self._read_evs[st.cuda_stream] = ev

    # ----------------------------------------------------------------- mutation
    def _grow(self, need: int):
        cap = self.X.shape[0]
        if need <= cap:
            return
        new = max(need, int(cap * 1.5) + 64)
        X = torch.zeros((new, self.dim), dtype=self.X.dtype, device=self.device)
        X[:self.n] = self.X[:self.n]
        s = torch.full((new,), -1, dtype=torch.int32, device=self.device)
        s[:self.n] = self.slots_t[:self.n]
        ids = np.zeros(new, dtype=np.int64)
        ids[:self.n] = self.ids[:self.n]
        ids_t = torch.zeros(new, dtype=torch.int64, device=self.device)
        ids_t[:self.n] = self.ids_t[:self.n]
        if self.device.type == "cuda":
            # the copies above read the old buffers on this stream: the allocator must not hand
            # them out again (to an allocation on their own stream) before those copies ran
            st = torch.cuda.current_stream(self.device)
            for old in (self.X, self.slots_t, self.ids_t):
                old.record_stream(st)
        self.X, self.slots_t, self.ids, self.ids_t = X, s, ids, ids_t

    def doc_slot(self, doc_id: str) -> int:
        e = self.docs.get(doc_id)
        if e is None:
            e = DocEntry(slot=len(self.slot_docs))
            self.docs[doc_id] = e
            self.slot_docs.append(doc_id)
        return e.slot

    def add(self, doc_id: str, ids: np.ndarray, vecs: torch.Tensor) -> tuple[int, int]:
        """Append the vectors of one document. ``vecs`` [n, d] (unit norm), any float dtype/device."""
        n = int(vecs.shape[0])
        if n == 0:
            self.doc_slot(doc_id)
            return (self.n, self.n)
        if vecs.shape[1] != self.dim:
            raise ValueError(f"vector dim {vecs.shape[1]} != index dim {self.dim}")
        with self.writing():
            slot = self.doc_slot(doc_id)
            s0 = self.n
            self._grow(s0 + n)
            self.X[s0:s0 + n] = vecs.to(device=self.device, dtype=self.X.dtype)
            self.slots_t[s0:s0 + n] = slot
            self.ids[s0:s0 + n] = np.asarray(ids, dtype=np.int64)
            self.ids_t[s0:s0 + n] = h2d(self.ids[s0:s0 + n], self.device)
            self.n = s0 + n
            e = self.docs[doc_id]
            e.ranges.append((s0, s0 + n))
            e.rows += n
            return (s0, s0 + n)

    def add_bulk(self, doc_ids: list[str], rows_per_doc: list[int], ids: np.ndarray, vecs: torch.Tensor):
        """Bulk load (benchmarks / snapshot restore): documents laid out back to back."""
        with self.writing():
            n = int(vecs.shape[0])
            s0 = self.n
            self._grow(s0 + n)
            self.X[s0:s0 + n] = vecs.to(device=self.device, dtype=self.X.dtype)
            self.ids[s0:s0 + n] = ids
            self.ids_t[s0:s0 + n] = h2d(np.asarray(ids, dtype=np.int64), self.device)
            slots = np.empty(n, dtype=np.int32)
            r = s0
            for d, k in zip(doc_ids, rows_per_doc):
                sl = self.doc_slot(d)
                slots[r - s0:r - s0 + k] = sl
                e = self.docs[d]
                e.ranges.append((r, r + k))
                e.rows += k
                r += k
            self.slots_t[s0:s0 + n] = h2d(slots, self.device)
            self.n = s0 + n

    def remove_doc(self, doc_id: str) -> int:
        """Drop a document's rows from search (rows become unreachable; compacted on snapshot)."""
        with self.writing():
            e = self.docs.get(doc_id)
            if e is None:
                return 0
            for a, b in e.ranges:
                self.slots_t[a:b] = -1
            n = e.rows
            e.ranges, e.rows = [], 0
            return n

    def remove_keys(self, doc_id: str, keys) -> int:
        """Drop the rows of ``doc_id`` whose external ids are in ``keys`` (per-chunk upsert: the
        reference's ``ON CONFLICT (chunk_id)``, postgres.go:197). Rows tracked by range (flat rows,
        IVF delta rows) have their ranges split around the dropped rows; rows tracked only by slot
        (IVF list-major rows) leave search through their slot. Returns the rows dropped."""
        keys = np.unique(np.asarray(keys, dtype=np.int64))
        with self.writing():
            e = self.docs.get(doc_id)
            if e is None or e.rows == 0 or keys.size == 0 or self.n == 0:
                return 0
            n = self.n
            kt = h2d(keys, self.device)
            s = self.slots_t[:n]
            sel = (s == e.slot) & torch.isin(self.ids_t[:n], kt)
            removed = int(sel.sum().item())
            if removed == 0:
                return 0
            s.masked_fill_(sel, -1)
            ranges = []
            for a, b in e.ranges:
                keep = ~np.isin(self.ids[a:b], keys)
                if keep.all():
                    ranges.append((a, b))
                    continue
                # maximal runs of kept rows
                edges = np.flatnonzero(np.diff(np.concatenate(([0], keep.view(np.int8), [0]))))
                ranges.extend((a + int(x), a + int(y)) for x, y in zip(edges[::2], edges[1::2]))
            e.ranges = ranges
            e.rows -= removed
            return removed

    def __len__(self):
        return self.n

    # ----------------------------------------------------------------- search
    def _ranges_for(self, doc_filters):
        ranges, off, maxrows = [], [0], 0
        for f in doc_filters:
            tot = 0
            for d in (self.docs if f is None else f):  # None = every document
                e = self.docs.get(d)
                if e is None:
                    continue
                for a, b in e.ranges:
                    ranges.append((a, b))
                    tot += b - a
            off.append(len(ranges))
            maxrows = max(maxrows, tot)
        return ranges, off, maxrows

    def search(self, q: torch.Tensor, k: int, min_sim: float, doc_filters: list[list[str]] | None = None):
        """q [Q, d] unit-norm -> (scores fp32 [Q, k], row idx int32 [Q, k]) on device; -inf / -1 padding.
        doc_filters: per-query list of document ids (None = all documents)."""
        Q = q.shape[0]
        q = q.to(device=self.device, dtype=self.X.dtype).contiguous()
        with self.reading():
            if self.n == 0 or Q == 0:
                return (torch.full((Q, k), float("-inf"), device=self.device),
                        torch.full((Q, k), -1, dtype=torch.int32, device=self.device))
            X = self.X[:self.n]
            if doc_filters is None:
                return self._dense(X, q, k, min_sim, self.slots_t[:self.n])
            ranges, off, maxrows = self._ranges_for(doc_filters)
            if maxrows == 0:
                return (torch.full((Q, k), float("-inf"), device=self.device),
                        torch.full((Q, k), -1, dtype=torch.int32, device=self.device))
            if maxrows * Q > 4 * self.n and self.dim % 32 == 0:
                # wide filters: one MFMA dense scan + bitmap beats per-query range scans
                return self._dense(X, q, k, min_sim, self.slots_t[:self.n], doc_filters)
            rt = h2d(np.asarray(ranges, dtype=np.int32).reshape(-1, 2), self.device)
            ot = h2d(np.asarray(off, dtype=np.int32), self.device)
            return self.ops.topk_ranges(X, q, rt, ot, k, min_sim, max_rows=maxrows)

    def _dense(self, X, q, k, min_sim, slots, doc_filters=None):
        """MFMA dense scan; doc filter as a bitmap over local doc slots. Removed rows (slot -1) map to
        a guard slot whose bit is never set."""
        Q = q.shape[0]
        nslots = len(self.slot_docs)
        guard = nslots
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
        bitmap = h2d(bm.view(np.int32), self.device)
        slots = torch.where(slots < 0, torch.full_like(slots, guard), slots).contiguous()
        return self.ops.topk_dense(X, q, k, min_sim, slots=slots, bitmap=bitmap)

    def gather_ids(self, rows: torch.Tensor) -> torch.Tensor:
        """Device: row indices (int32, -1 = none) -> external ids (int64, -1 = none). Indices are
        clamped into the id table before the gather (a bad row index must never read outside it)."""
        with self.reading():
            r = rows.long()
            ok = (r >= 0) & (r < self.n)
            return torch.where(ok, self.ids_t[r.clamp(0, max(0, self.n - 1))], torch.full_like(r, -1))

    def search_ids(self, q: torch.Tensor, k: int, min_sim: float, doc_filters=None):
        """search + gather_ids as ONE read: (scores fp32 [Q, k], external ids int64 [Q, k]) from the
        same committed state of the shard."""
        with self.reading():
            s, rows = self.search(q, k, min_sim, doc_filters)
            return s, self.gather_ids(rows)

    def row_ids(self, rows: np.ndarray) -> np.ndarray:
        out = np.full(rows.shape, -1, dtype=np.int64)
        m = rows >= 0
        out[m] = self.ids[rows[m]]
        return out

    # ----------------------------------------------------------------- snapshot
    def live_rows_by_doc(self):
        """(rows grouped by document, [(doc_id, n_rows)]) for snapshots (removed docs dropped)."""
        docs, rows = [], []
        for d, e in self.docs.items():
            n = 0
            for a, b in e.ranges:
                rows.append((a, b))
                n += b - a
            docs.append((d, n))
        sel = np.concatenate([np.arange(a, b) for a, b in rows]) if rows else np.zeros(0, dtype=np.int64)
        return sel.astype(np.int64), docs

    def state_dict(self) -> dict:
        with self.reading():
            live = []
            for d, e in self.docs.items():
                for a, b in e.ranges:
                    live.append((d, a, b))
            return {"dim": self.dim, "live": live, "X": self.X[:self.n].cpu(), "ids": self.ids[:self.n].copy()}

    def nbytes(self) -> int:
        return self.n * self.dim * self.X.element_size()


def bytes_per_row(dim: int) -> int:
    return dim * 2 + 4


def rows_for_budget(dim: int, gbytes: float) -> int:
    return int(gbytes * 1e9 // bytes_per_row(dim))


def _pad64(n: int) -> int:
    return int(math.ceil(n / 64) * 64)
