"""Sharded vector search as rounds across every rank, decoupled from the decode schedulers.

The engine serves as independent data-parallel replicas (one per TP group, each with its own RPC
endpoint and continuous-batching scheduler, no per-tick collective; engine/server.py), the way the
reference scales its agents (docker-compose.yml:84-85,105-106; internal/queue/nats.go:40-51). The
vector index, though, is sharded over ALL ranks (a document lives on rank hash(doc) % N), so a
search needs every shard. That exchange runs here, on a thread and HIP stream of its own on every
rank, so a search never waits for any replica's decode tick or admission prefill:

    round:  all-gather (rows, k, stop) per rank            gloo, 24 B per rank (the poll)
            all-gather filters / thresholds of the rows     gloo, msgpack bytes
            C2 all-gather of the query vectors              data group (RCCL on GPUs, over xGMI)
            fused scan + doc filter + floor + top-k on the local shard (vecsearch.hip)
            C1 all-gather of packed (score, id) top-k       data group (RCCL)
            topk_merge kernel -> each rank resolves the requests it submitted

A rank with nothing to search still joins each round (its rows = 0) — a poll every ``poll_s``
(1 ms while searches are flowing, ``idle_poll_s`` after a second without any). Results equal the
single-index exact search (filter and floor applied before each shard's top-k; k / floor
per request: the round runs max k / min floor and each request is cut back, which is exact because
every row above a request's floor ranks above every row below it).
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from .dist import pack_scores_ids, unpack_scores_ids


def merge_shard_topk(ops, S: torch.Tensor, G: torch.Tensor, k: int):
    """Per-shard top-k lists S / G [W, B, k] (score fp32, id int64, -1 = none) -> the global top-k
    [B, k] with the topk_merge kernel (candidate ids = positions shard * k + j, so ties resolve
    deterministically to the lower shard / rank, then the lower position)."""
    W, B, _ = S.shape
    pos = torch.arange(W * k, dtype=torch.int32, device=S.device).view(W, 1, k).expand(W, B, k).contiguous()
    pos = torch.where(G >= 0, pos, torch.full_like(pos, -1))
    S = torch.where(G >= 0, S, torch.full_like(S, float("-inf"))).contiguous()
    ms, mp = ops.topk_merge(S, pos, k)
    flatG = G.permute(1, 0, 2).reshape(B, W * k)
    mid = torch.where(mp >= 0, flatG.gather(1, mp.clamp_min(0).long()), torch.full_like(flatG[:, :k], -1))
    return ms, mid


class _Req:
    __slots__ = ("vecs", "k", "thr", "filters", "fut")

    def __init__(self, vecs, k, thr, filters, fut):
        self.vecs, self.k, self.thr, self.filters, self.fut = vecs, k, thr, filters, fut


class SearchPlane:
    """One per rank. ``submit`` from any thread; results arrive as concurrent futures."""

    def __init__(self, index, rank: int = 0, world: int = 1, ctrl_group=None, data_group=None, device=None,
                 poll_s: float = 0.001, idle_poll_s: float = 0.005, max_rows: int = 1024, stream=None):
        self.index, self.rank, self.world = index, rank, world
        self.ctrl_group, self.data_group = ctrl_group, data_group
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.poll_s, self.idle_poll_s, self.max_rows = poll_s, idle_poll_s, max_rows
        self.q: collections.deque = collections.deque()
        self.cv = threading.Condition()
        self.stream = stream  # None: a high-priority stream created by the plane thread
        self.write_event = None
        self._stop = False
        self._thread = None
        self._last_active = 0.0
        self.healthy = True
        self.error = ""
        self.stats = {"rounds": 0, "empty_rounds": 0, "queries": 0, "busy_s": 0.0}

    # ------------------------------------------------------------------ public
    def submit(self, vecs: np.ndarray, k: int, min_sim: float, filters=None) -> cf.Future:
        """vecs [n, d]; filters: None, or a list of n document-id lists (or one list for all rows)."""
        vecs = np.ascontiguousarray(vecs, dtype=np.float32).reshape(-1, self.index.dim)
        n = vecs.shape[0]
        if filters is not None:
            if len(filters) == 1 and n != 1:
                filters = list(filters) * n
            if len(filters) != n:
                raise ValueError("search: one document filter per query row (or one for all rows)")
            filters = [None if f is None else list(f) for f in filters]
        fut: cf.Future = cf.Future()
        if not self.healthy:
            fut.set_exception(RuntimeError(f"search plane down: {self.error}"))
            return fut
        with self.cv:
            self.q.append(_Req(vecs, int(k), float(min_sim), filters, fut))
            self.cv.notify()
        return fut

    def note_write(self) -> None:
        """Called by the thread that mutated the index (after the mutation was enqueued on its
        stream): the next round's scan waits for it on the device."""
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self.write_event = ev

    def start(self) -> "SearchPlane":
        self._thread = threading.Thread(target=self._run, name=f"search-plane-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def stop(self, timeout: float = 30.0) -> None:
        """Leave the plane: this rank's next round carries the stop flag, and every rank exits the
        round in which it sees one (so the whole engine stops searching together)."""
        with self.cv:
            self._stop = True
            self.cv.notify()
        if self._thread is not None:
            self._thread.join(timeout)

    # ------------------------------------------------------------------ rounds
    def _run(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        try:
            while self._round():
                pass
        except Exception as e:  # noqa: BLE001 - a dead peer / collective timeout: fail loudly, stop
            self.healthy = False
            self.error = repr(e)
        finally:
            self._fail_pending(RuntimeError(f"search plane stopped{': ' + self.error if self.error else ''}"))

    def _fail_pending(self, exc):
        with self.cv:
            while self.q:
                r = self.q.popleft()
                if not r.fut.done():
                    r.fut.set_exception(exc)

    def _take(self) -> list[_Req]:
        out, n = [], 0
        with self.cv:
            while self.q and (not out or n + self.q[0].vecs.shape[0] <= self.max_rows):
                r = self.q.popleft()
                out.append(r)
                n += r.vecs.shape[0]
        return out

    def _round(self) -> bool:
        if self.world == 1:
            with self.cv:
                while not self.q and not self._stop:
                    self.cv.wait(0.5)
                if self._stop and not self.q:
                    return False
            take = self._take()
            if take:
                self._serve(take, None)
            return True
        take = self._take()
        n = sum(r.vecs.shape[0] for r in take)
        hdr = torch.tensor([n, max((r.k for r in take), default=0), 1 if self._stop else 0], dtype=torch.int64)
        allh = torch.empty(self.world * 3, dtype=torch.int64)
        dist.all_gather_into_tensor(allh, hdr, group=self.ctrl_group)
        allh = allh.view(self.world, 3)
        if int(allh[:, 2].max()) > 0:
            for r in take:
                if not r.fut.done():
                    r.fut.set_exception(RuntimeError("search plane stopping"))
            return False
        if int(allh[:, 0].sum()) == 0:
            self.stats["empty_rounds"] += 1
            idle = time.monotonic() - self._last_active > 1.0
            with self.cv:
                if not self.q and not self._stop:
                    self.cv.wait(self.idle_poll_s if idle else self.poll_s)
            return True
        self._last_active = time.monotonic()
        self._serve(take, allh)
        return True

    def _serve(self, take: list[_Req], allh):
        t0 = time.perf_counter()
        idx, dev = self.index, self.index.device
        d = idx.dim
        stream_ctx = torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()
        # the scan kernels' scratch must not be the GPU thread's: its decode graph captured that
        # workspace's pointer and runs concurrently with this thread (ops/kernels.py workspace_role)
        ws_ctx = _nullctx()
        if dev.type == "cuda":
            from ..ops.kernels import workspace_role
            ws_ctx = workspace_role("search")
        with stream_ctx, ws_ctx:
            if self.write_event is not None and self.stream is not None:
                self.stream.wait_event(self.write_event)
            rows = [r.vecs.shape[0] for r in take]
            mine_q = np.concatenate([r.vecs for r in take]) if take else np.zeros((0, d), np.float32)
            mine_f = [f for r in take for f in (r.filters if r.filters is not None else [None] * r.vecs.shape[0])]
            mine_thr = [r.thr for r in take for _ in range(r.vecs.shape[0])]
            if allh is None:  # one rank: the local shard is the whole index
                counts, K = [len(mine_q)], max(r.k for r in take)
                filters, thr_all, Q = mine_f, mine_thr, torch.from_numpy(mine_q).to(dev)
            else:
                from .dist import all_gather_bytes
                from ..engine.rpc import dumps, loads
                counts = [int(x) for x in allh[:, 0].tolist()]
                K = int(allh[:, 1].max())
                parts = [loads(p) for p in all_gather_bytes(dumps([mine_f, mine_thr]), "cpu", self.ctrl_group)]
                filters = [f for fs, _ in parts for f in fs]
                thr_all = [t for _, ts in parts for t in ts]
                maxn = max(counts)
                pad = torch.zeros((maxn, d), dtype=torch.float32, device=self._data_dev())
                if len(mine_q):
                    pad[:len(mine_q)] = torch.from_numpy(mine_q).to(pad.device)
                allq = torch.empty((self.world * maxn, d), dtype=torch.float32, device=pad.device)
                dist.all_gather_into_tensor(allq, pad, group=self.data_group)             # C2
                sel = torch.cat([torch.arange(r * maxn, r * maxn + c) for r, c in enumerate(counts)])
                Q = allq.index_select(0, sel.to(allq.device)).to(dev)
            thr = float(min(thr_all))
            nofilter = all(f is None for f in filters)
            with idx.lock:
                s, rowsel = idx.search(Q, K, thr, None if nofilter else filters)
                gid = idx.gather_ids(rowsel)
                if self.stream is not None:
                    self.stream.synchronize()  # the scan has read the shard before a writer may touch it
            if allh is None:
                ms, mid = s, gid
            else:
                P = pack_scores_ids(s, gid).to(self._data_dev())
                allp = torch.empty((self.world,) + tuple(P.shape), dtype=P.dtype, device=P.device)
                dist.all_gather_into_tensor(allp.view(-1, *P.shape[1:]), P, group=self.data_group)  # C1
                S, G = unpack_scores_ids(allp.to(dev))                                       # [W, Qtot, K]
                o = sum(counts[:self.rank])
                S, G = S[:, o:o + counts[self.rank]].contiguous(), G[:, o:o + counts[self.rank]].contiguous()
                ms, mid = merge_shard_topk(idx.ops, S, G, K) if counts[self.rank] else (S[0], G[0])
            ms, mid = ms.float().cpu().numpy(), mid.cpu().numpy()
        o = 0
        for r, n in zip(take, rows):
            sc, ky = ms[o:o + n, :r.k].copy(), mid[o:o + n, :r.k].copy()
            drop = ~(sc >= r.thr)
            sc[drop], ky[drop] = -np.inf, -1
            if not r.fut.done():
                r.fut.set_result((sc, ky))
            o += n
        self.stats["rounds"] += 1
        self.stats["queries"] += sum(rows)
        self.stats["busy_s"] += time.perf_counter() - t0

    def _data_dev(self):
        if self.data_group is not None and dist.get_backend(self.data_group) == "gloo":
            return torch.device("cpu")
        return self.index.device if self.index.device.type == "cuda" else torch.device("cpu")


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
