"""Serving search over RCCL (SEARCH_TRANSPORT=rccl): lock-step rounds of all-gathers over xGMI.

The default serving transport (parallel/search_plane.py) routes each search point to point to the
shards that own its documents, so a dead rank fails only the searches that touch its shard. This is
the collective alternative the north star names: every search of every rank travels in ONE world-wide
round, the query rows and the per-shard top-k lists as two RCCL all-gathers.

    round thread (one per rank, its own HIP stream and scan workspace), forever:
      take this rank's queued searches (<= max_rows rows)
      M   all_gather_object over the gloo control group: (rows, k, floor, filters, stop) per rank
          every rank idle -> wait for work, next round; the wait backs off from idle_s to
          idle_max_s (x2 per idle round), so an idle world does <= 1 / idle_max_s control
          gathers per second per rank, and a search that arrives wakes its own rank at once
          (its peers join within idle_max_s)
      C2  all-gather of the zero-padded query rows              [W * B, d]       (RCCL)
          ONE fused scan + doc filter + floor + top-k of every rank's rows on the local shard
      C1  all-gather of the packed (score, id) top-k lists      [W, W * B, k, 2] (RCCL)
          device merge (topk_merge kernel) of this rank's rows -> each search's futures

Exactness: a document lives on one shard and each shard applies the filter and the floor before
its top-k, so the merge equals the single-index search (the same argument, and the same tie order —
lower rank, then lower position — as the point-to-point plane and ShardedIndex). Searches with
different k / floor share a round at max k / min floor and are cut back after the merge (exact: a
row above a search's floor ranks above every row below it). Padded rows filter on no document.

What it trades (why it is not the default): a round is a rendezvous of every rank, so one hung or
dead rank stops search on all of them (an RCCL communicator cannot lose a member). The control
all-gather carries the group's timeout: when it expires the transport reports itself down (health:
every peer in ``shards_down``) and fails its searches, instead of hanging them. It also assumes no
other thread of the process drives RCCL concurrently: the engine allows it only with TP_SIZE=1, where
the GPU thread issues no collectives (engine_main checks).
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import logging
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from .dist import all_gather_rows, pack_scores_ids, unpack_scores_ids
from .search_plane import _nullctx, merge_shard_topk

_log = logging.getLogger(__name__)
_SCAN_FAILED = -2  # id marking every entry of a shard's lists whose scan failed in a round


class _Pending:
    __slots__ = ("vecs", "k", "thr", "filters", "fut", "deadline")

    def __init__(self, vecs, k, thr, filters, fut, deadline):
        self.vecs, self.k, self.thr, self.filters, self.fut, self.deadline = vecs, k, thr, filters, fut, deadline


def _settle(fut: cf.Future, result=None, exc=None) -> None:
    """Resolve a future once (the timer may have failed it already)."""
    try:
        if exc is not None:
            fut.set_exception(exc)
        else:
            fut.set_result(result)
    except cf.InvalidStateError:
        pass


class CollectiveSearchPlane:
    """The search-plane interface (``submit`` / ``health`` / ``stats`` / ``stop``) over lock-step
    collective rounds. Every rank of ``ctrl_group`` / ``data_group`` must construct and start one."""

    def __init__(self, index, rank: int = 0, world: int = 1, data_group=None, ctrl_group=None, device=None,
                 stream=None, timeout_s: float = 30.0, max_rows: int = 1024, idle_s: float = 0.002,
                 idle_max_s: float = 0.05):
        self.index, self.rank, self.world = index, rank, max(1, world)
        self.data_group, self.ctrl_group = data_group, ctrl_group
        self.device = torch.device(device) if device is not None else getattr(index, "device", torch.device("cpu"))
        self.stream = stream
        self.timeout_s, self.max_rows, self.idle_s = timeout_s, max_rows, idle_s
        self.idle_max_s = max(idle_s, idle_max_s)
        self.pending: collections.deque = collections.deque()
        self.inflight: list[_Pending] = []
        self.cv = threading.Condition()
        self._stop = False
        self._threads: list[threading.Thread] = []
        self.error = ""
        self.stopped_by = None
        self.stats = {"searches": 0, "rounds": 0, "idle_rounds": 0, "idle_gathers": 0, "rows": 0, "round_rows": 0,
                      "busy_s": 0.0, "failed": 0, "expired": 0, "local_failures": 0, "transport": "rccl" if self._nccl() else "gloo"}

    def _nccl(self) -> bool:
        return (self.world > 1 and dist.is_initialized()
                and dist.get_backend(self.data_group) == "nccl")

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "CollectiveSearchPlane":
        for fn, name in ((self._round_loop, "round"), (self._timer, "timer")):
            t = threading.Thread(target=fn, name=f"cplane-{name}-{self.rank}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self, timeout: float = 10.0) -> None:
        """Ends the rounds on EVERY rank (the stop travels in the next round's control gather)."""
        with self.cv:
            self._stop = True
            self.cv.notify_all()
        for t in self._threads:
            if t is not threading.current_thread():
                t.join(timeout)
        self._fail_all(RuntimeError("search transport stopped"))

    @property
    def healthy(self) -> bool:
        return not self._stop and not self.error and all(t.is_alive() for t in self._threads)

    def health(self) -> dict:
        if self.healthy:
            return {"ok": True, "shards_down": [], "errors": {}}
        why = self.error or (f"stopped by rank {self.stopped_by}" if self.stopped_by is not None else "stopped")
        down = [r for r in range(self.world) if r != self.rank]
        return {"ok": False, "shards_down": down, "errors": {str(r): why for r in down}}

    # ------------------------------------------------------------------ submit
    def submit(self, vecs, k: int, min_sim: float, filters=None) -> cf.Future:
        """vecs [n, d]; filters None or one document-id list per row (or one for all rows).
        Future -> (scores fp32 [n, k], external ids int64 [n, k]), -inf / -1 padded."""
        vecs = np.ascontiguousarray(vecs, dtype=np.float32).reshape(-1, self.index.dim)
        n, k, thr = vecs.shape[0], int(k), float(min_sim)
        if filters is not None:
            if len(filters) == 1 and n != 1:
                filters = list(filters) * n
            if len(filters) != n:
                raise ValueError("search: one document filter per query row (or one for all rows)")
            filters = [None if f is None else [str(d) for d in f] for f in filters]
        if not 0 < k <= 1024:
            raise ValueError(f"bad k {k}")
        fut: cf.Future = cf.Future()
        if not self.healthy and self._threads or self._stop:
            fut.set_exception(RuntimeError(f"search transport down: {self.health()['errors'] or 'stopped'}"))
            return fut
        self.stats["searches"] += 1
        if n == 0:
            fut.set_result((np.full((0, k), -np.inf, np.float32), np.full((0, k), -1, np.int64)))
            return fut
        with self.cv:
            self.pending.append(_Pending(vecs, k, thr, filters, fut, time.monotonic() + self.timeout_s))
            self.cv.notify()
        return fut

    # ------------------------------------------------------------------ rounds
    def _take(self) -> list[_Pending]:
        out, n, now = [], 0, time.monotonic()
        with self.cv:
            while self.pending and (not out or n + self.pending[0].vecs.shape[0] <= self.max_rows):
                p = self.pending.popleft()
                if p.fut.done():
                    continue  # the timer failed it while queued
                if now > p.deadline:
                    self.stats["expired"] += 1
                    _settle(p.fut, exc=TimeoutError("search expired before its round"))
                    continue
                out.append(p)
                n += p.vecs.shape[0]
            self.inflight = list(out)
        return out

    def _round_loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        take: list[_Pending] = []
        wait = self.idle_s
        try:
            while True:
                with self.cv:
                    if not self.pending and not self._stop:
                        self.cv.wait(wait)
                    stopping = self._stop
                take = [] if stopping else self._take()
                rows = sum(p.vecs.shape[0] for p in take)
                filters = None
                if any(p.filters is not None for p in take):
                    filters = [f for p in take for f in (p.filters if p.filters is not None else [None] * p.vecs.shape[0])]
                meta = {"n": rows, "k": max((p.k for p in take), default=0),
                        "thr": min((p.thr for p in take), default=float("inf")), "filters": filters,
                        "stop": stopping}
                metas = [meta]
                if self.world > 1:
                    metas = [None] * self.world
                    dist.all_gather_object(metas, meta, group=self.ctrl_group)                     # M
                stop_ranks = [r for r, m in enumerate(metas) if m["stop"]]
                if stop_ranks:
                    self.stopped_by = stop_ranks[0]
                    self._stop = True
                    exc = RuntimeError(f"search transport stopped by rank {stop_ranks[0]}")
                    for p in take:
                        _settle(p.fut, exc=exc)
                    # and every search still queued here (submitted during the gather, or left out
                    # by max_rows): no round will run them
                    self._fail_all(exc)
                    break
                if max(m["n"] for m in metas) == 0:
                    self.stats["idle_rounds"] += 1
                    self.stats["idle_gathers"] += 1
                    wait = min(self.idle_max_s, wait * 2)
                    continue
                wait = self.idle_s
                self._round(take, metas)
                take = []
                with self.cv:
                    self.inflight = []
        except Exception as e:  # noqa: BLE001 - a failed collective ends the transport on this rank
            self.error = f"{type(e).__name__}: {e}"
            _log.error("search transport round failed on rank %d: %s", self.rank, self.error, exc_info=True)
            for p in take:
                _settle(p.fut, exc=RuntimeError(f"search transport down: {self.error}"))
            self._fail_all(RuntimeError(f"search transport down: {self.error}"))

    def _round(self, take: list[_Pending], metas: list[dict]):
        t0 = time.perf_counter()
        W, idx, dev = self.world, self.index, self.index.device
        live = [m for m in metas if m["n"] > 0]
        B = max(m["n"] for m in metas)
        K = max(m["k"] for m in live)
        thr = min(m["thr"] for m in live)
        n = metas[self.rank]["n"]
        Q = np.zeros((B, idx.dim), dtype=np.float32)
        local_err = None  # a failure of this rank's own work fails only its searches of this round:
        # the rank still joins every collective (its peers are already in them) and the next rounds
        try:
            if n:
                Q[:n] = np.concatenate([p.vecs for p in take])
        except Exception as e:  # noqa: BLE001
            local_err = e
        # every rank's rows in rank order, B per rank; padded rows filter on no document
        if all(m["n"] == B and m["filters"] is None for m in metas):
            filters_all = None
        else:
            filters_all = []
            for m in metas:
                f = m["filters"] if m["filters"] is not None else [None] * m["n"]
                filters_all.extend(list(f) + [[]] * (B - m["n"]))
        stream_ctx = torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()
        ws_ctx = _nullctx()
        if dev.type == "cuda":
            from ..ops.kernels import workspace_role
            # not the GPU thread's scratch (its decode graph holds it), nor a point-to-point plane's
            # scan worker's (a process may run both: bench.py's serving_search block)
            ws_ctx = workspace_role("search_rounds")
        with stream_ctx, ws_ctx:
            q = torch.from_numpy(Q).to(dev)
            qs = all_gather_rows(q, self.data_group) if W > 1 else q                       # C2
            scan_err = None
            try:
                s, g = idx.search_ids(qs, K, thr, filters_all)
            except Exception as e:  # noqa: BLE001 - this shard's scan failed: the round goes on
                # (the collectives stay in lock-step); every id of its lists carries the failure
                scan_err = e
                _log.error("search shard %d: scan failed in a round: %r", self.rank, e)
                s = torch.full((W * B, K), float("-inf"), device=qs.device)
                g = torch.full((W * B, K), _SCAN_FAILED, dtype=torch.int64, device=qs.device)
            if W > 1:
                P = all_gather_rows(pack_scores_ids(s, g), self.data_group)                 # C1
                S, G = unpack_scores_ids(P)
                S = S.reshape(W, W * B, K)
                G = G.reshape(W, W * B, K)
                if n == 0:  # an idle rank joins the collectives and has nothing to merge
                    return self._count(0, W * B, t0)
            # past the collectives: everything below is this rank's own (merge, copy back, settle)
            try:
                if local_err is not None:
                    raise local_err
                if W > 1:
                    mine = slice(self.rank * B, self.rank * B + n)
                    failed = [r for r in range(W) if bool((G[r, mine] == _SCAN_FAILED).any())]
                    if failed:
                        exc = RuntimeError(f"search shards {failed} failed their scan in this round")
                        for p in take:
                            _settle(p.fut, exc=exc)
                        self.stats["failed"] += len(take)
                        return self._count(n, W * B, t0)
                    s, g = merge_shard_topk(idx.ops, S[:, mine].contiguous(), G[:, mine].contiguous(), K)
                else:
                    if scan_err is not None:
                        for p in take:
                            _settle(p.fut, exc=RuntimeError(f"search shard scan failed: {scan_err!r}"))
                        return self._count(n, W * B, t0)
                    s, g = s[:n], g[:n]
                s, g = s.float().cpu().numpy(), g.cpu().numpy()
            except Exception as e:  # noqa: BLE001
                _log.error("search rank %d: local merge failed in a round: %r", self.rank, e)
                self.stats["local_failures"] += 1
                for p in take:
                    _settle(p.fut, exc=RuntimeError(f"search round failed on rank {self.rank}: {e!r}"))
                return self._count(n, W * B, t0)
        o = 0
        for p in take:
            m = p.vecs.shape[0]
            sc, ky = s[o:o + m, :p.k].copy(), g[o:o + m, :p.k].copy()
            drop = ~(sc >= p.thr)
            sc[drop], ky[drop] = -np.inf, -1
            _settle(p.fut, (sc, ky))
            o += m
        self._count(n, W * B, t0)

    def _count(self, n: int, round_rows: int, t0: float) -> None:
        self.stats["rounds"] += 1
        self.stats["rows"] += n
        self.stats["round_rows"] += round_rows
        self.stats["busy_s"] += time.perf_counter() - t0

    def _timer(self):
        """Fail searches past their deadline, queued or in a round that does not come back (a hung
        peer holds the collective)."""
        while not self._stop and not self.error:
            time.sleep(0.1)
            now = time.monotonic()
            with self.cv:
                late = [p for p in list(self.pending) + list(self.inflight) if now > p.deadline and not p.fut.done()]
            for p in late:
                self.stats["failed"] += 1
                _settle(p.fut, exc=TimeoutError(f"search round did not complete within {self.timeout_s:.0f} s"))

    def _fail_all(self, exc):
        with self.cv:
            ps, self.pending = list(self.pending) + list(self.inflight), collections.deque()
            self.inflight = []
        for p in ps:
            _settle(p.fut, exc=exc)
