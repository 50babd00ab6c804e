"""Sharded vector search routed to the owner shards, point to point, with failures isolated per shard.

The engine serves as independent data-parallel replicas (one per TP group, each with its own RPC
endpoint and continuous-batching scheduler; engine/server.py), the way the reference scales its
agents (docker-compose.yml:84-85,105-106; internal/queue/nats.go:40-51). The vector index is
sharded over ALL ranks: a document's rows live on rank ``owner_of(doc_id, world)``. Every search in
the reference is filtered by a required, non-empty document list (cmd/query/main.go:22,
internal/store/postgres.go:239), so a search only needs the shards that own its filter's documents:

    submit(q, k, floor, filters)        any thread, any rank
      route: rows -> owner ranks of their filter documents (no filter: every rank)
      local part  -> this rank's scan worker                        (no socket)
      remote part -> the owner's shard server: one msgpack frame    (TCP, persistent connection)
    shard server (every rank): a scan worker thread with its own HIP stream and kernel workspace
      drains every queued part (local and remote) as ONE fused scan + doc filter + floor + top-k
      launch on the local shard (vecsearch.hip), replies [m, k] (score, external id) per part
    merge on the submitter: per row, the owners' top-k lists -> the global top-k (ties: lower
      rank, then lower position — the order of the all-gather merge of ShardedIndex)

Why not a collective here. A collective round (the previous design, and ``ShardedIndex`` for
lock-step batch search) makes every search a world-wide rendezvous: every rank polls, an idle
rank still joins every round, and ONE dead or hung rank stops search for every replica, because an
RCCL communicator cannot lose a member. The reference's replicas fail independently. Here a search
waits only for the shards it reads: a dead rank fails the searches that touch its documents (the
health RPC names it) and nothing else; a restarted rank is reconnected on the next request. The
bytes are tiny (a 768-d fp32 query is 3 KB, a top-5 reply 60 B) and the hop is host TCP on one
node (~30-60 us), against a 15-20 ms question path. And it takes the search traffic off RCCL
altogether: RCCL is issued by one thread per process (the GPU thread: TP all-reduces above the
IPC limit, replica gathers), so no two threads ever drive two communicators concurrently.

Exactness: the doc filter and the similarity floor are applied inside each shard BEFORE its top-k,
and a document lives on exactly one shard, so the merged result equals the single-index exact
search. Requests with different k / floor share a scan (max k, min floor; each part is cut back,
which is exact because every row above a part's floor ranks above every row below it).
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import hashlib
import queue
import socket
import struct
import threading
import time

import numpy as np
import torch


def owner_of(doc_id: str, world: int) -> int:
    """The rank whose shard holds ``doc_id``'s rows (stable across processes: blake2b, not hash())."""
    return int.from_bytes(hashlib.blake2b(doc_id.encode(), digest_size=8).digest(), "little") % max(1, world)


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


def merge_host(parts, n: int, k: int, world: int, thr: float):
    """parts: {rank: (row index array [m], scores [m, k'], keys [m, k'])} -> (scores [n, k] fp32,
    keys [n, k] int64), -inf / -1 padded, floor applied. Ties: lower rank, then lower position."""
    S = np.full((n, world * k), -np.inf, dtype=np.float32)
    G = np.full((n, world * k), -1, dtype=np.int64)
    for r, (rows, s, g) in parts.items():
        kk = min(k, s.shape[1])
        S[rows, r * k:r * k + kk] = s[:, :kk]
        G[rows, r * k:r * k + kk] = g[:, :kk]
    S[G < 0] = -np.inf
    order = np.argsort(-S, axis=1, kind="stable")[:, :k]
    sc = np.take_along_axis(S, order, 1)
    ky = np.take_along_axis(G, order, 1)
    drop = ~(sc >= thr)
    sc[drop], ky[drop] = -np.inf, -1
    return sc, ky


# --------------------------------------------------------------------------- framing
def _send_frame(sock, obj) -> None:
    from ..engine.rpc import pack
    sock.sendall(pack(obj))


def _recv_exact(sock, n: int, stopped=None) -> bytes:
    """n bytes from ``sock``. A socket with a timeout (the requester side: its timeout bounds SENDS)
    keeps waiting through idle timeouts, the partial frame kept, until ``stopped()``."""
    buf = bytearray()
    while len(buf) < n:
        try:
            b = sock.recv(n - len(buf))
        except socket.timeout:
            if stopped is not None and stopped():
                raise ConnectionError("search plane stopped") from None
            continue
        if not b:
            raise ConnectionError("peer closed the connection")
        buf += b
    return bytes(buf)


def _recv_frame(sock, stopped=None):
    from ..engine.rpc import unpack
    n = struct.unpack(">I", _recv_exact(sock, 4, stopped))[0]
    if n > (256 << 20):
        raise ConnectionError(f"oversized search frame ({n} B)")
    return unpack(_recv_exact(sock, n, stopped))


class ShardUnavailable(RuntimeError):
    pass


_REPLY_BACKLOG = 4096  # queued replies per requester connection before the shard drops it
_SEND_BACKLOG = 1024   # queued request frames per peer before new parts fail fast
_QUEUED_ROWS_MAX = 1 << 16  # query rows queued on a shard before it refuses more (overload)


class _Job:
    """One part of a search on the local shard: rows [m, d] + per-row filters, and where the answer
    goes (``reply(scores, keys)`` / ``fail(exc)``); ``deadline`` (monotonic s, None = none): past it
    the requester has given up, so the scan worker drops the job instead of scanning it."""
    __slots__ = ("vecs", "k", "thr", "filters", "reply", "fail", "deadline")

    def __init__(self, vecs, k, thr, filters, reply, fail, deadline=None):
        self.vecs, self.k, self.thr, self.filters, self.reply, self.fail = vecs, k, thr, filters, reply, fail
        self.deadline = deadline


class _Search:
    """A submitted search waiting for its parts."""
    __slots__ = ("n", "k", "thr", "left", "parts", "fut", "deadline", "lock", "ranks")

    def __init__(self, n, k, thr, ranks, fut, deadline):
        self.n, self.k, self.thr, self.fut, self.deadline = n, k, thr, fut, deadline
        self.ranks = set(ranks)
        self.left = len(self.ranks)
        self.parts: dict = {}
        self.lock = threading.Lock()


class _Peer:
    """Client side of one remote shard: a persistent connection, its writer and reader threads, the
    pending parts. ``send`` never blocks its caller (the engine's event loop): it queues the frame
    for the writer thread, which connects (bounded by connect_timeout_s) and sends (bounded by
    send_timeout_s: a peer that accepts but stops reading is marked down when its receive buffer
    stays full that long). A failed connection fails only its own pending parts; the next request
    reconnects (at most once per ``retry_s``), so a restarted rank rejoins without coordination."""

    def __init__(self, plane, rank: int, addr):
        self.plane, self.rank, self.addr = plane, rank, tuple(addr)
        self.sock = None
        self.lock = threading.Lock()   # sock / pending (the reader takes it per reply)
        self.q: queue.Queue = queue.Queue(maxsize=_SEND_BACKLOG)
        self.writer = None
        self.pending: dict = {}
        self.down_since = None
        self.last_try = 0.0
        self.error = ""

    def _connect(self):
        now = time.monotonic()
        if self.down_since is not None and now - self.last_try < self.plane.retry_s:
            raise ShardUnavailable(f"search shard {self.rank} unavailable: {self.error}")
        self.last_try = now
        try:
            s = socket.create_connection(self.addr, timeout=self.plane.connect_timeout_s)
            s.settimeout(self.plane.send_timeout_s)  # bounds every sendall (the reader rides idle timeouts)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        except OSError as e:
            self.down_since = self.down_since or now
            self.error = repr(e)
            raise ShardUnavailable(f"search shard {self.rank} unavailable: {e!r}") from e
        self.sock = s
        self.down_since, self.error = None, ""
        threading.Thread(target=self._read_loop, args=(s,), name=f"plane-peer-{self.rank}", daemon=True).start()

    def send(self, rid: int, msg: dict, on_reply, on_fail, deadline: float | None = None):
        """Queue one request frame (never blocks: a full backlog fails the part at once).
        ``deadline`` (monotonic s): the search's own; a frame still queued past it is dropped, and
        the frame carries what is left of it as its ``ttl`` (the shard then expires the part on time
        however long it waited in this backlog)."""
        with self.lock:
            if self.writer is None:
                self.writer = threading.Thread(target=self._write_loop, name=f"plane-send-{self.rank}", daemon=True)
                self.writer.start()
        try:
            self.q.put_nowait((rid, msg, on_reply, on_fail, deadline))
        except queue.Full:
            on_fail(ShardUnavailable(f"search shard {self.rank}: {_SEND_BACKLOG} requests already queued"))

    def _write_loop(self):
        while not self.plane._stop:
            try:
                item = self.q.get(timeout=0.5)
            except queue.Empty:
                continue
            rid, msg, on_reply, on_fail, deadline = item
            if self.plane._stop:
                on_fail(RuntimeError("search plane stopped"))
                continue
            if deadline is not None:
                left = deadline - time.monotonic()
                if left <= 0:
                    self.plane.stats["expired"] += 1
                    on_fail(TimeoutError(f"search part for shard {self.rank} expired in the send backlog"))
                    continue
                msg["ttl"] = left
            sock = None
            try:
                with self.lock:
                    if self.sock is None:
                        self._connect()
                    self.pending[rid] = (on_reply, on_fail)
                    sock = self.sock
                # outside the lock: a send blocked on a slow shard's full receive buffer never holds
                # up the reader thread that delivers this peer's replies
                _send_frame(sock, msg)
            except ShardUnavailable as e:
                on_fail(e)
            except OSError as e:  # incl. socket.timeout: the shard stopped reading
                self._down(sock, e)
            except Exception as e:  # noqa: BLE001 - e.g. an unserialisable request: fails this part only
                with self.lock:
                    self.pending.pop(rid, None)
                on_fail(e)

    def _read_loop(self, sock):
        try:
            while True:
                msg = _recv_frame(sock, stopped=lambda: self.plane._stop or self.sock is not sock)
                with self.lock:
                    cb = self.pending.pop(msg.get("id"), None)
                if cb is None:
                    continue
                if "error" in msg:
                    cb[1](RuntimeError(f"search shard {self.rank}: {msg['error']}"))
                else:
                    cb[0](msg["scores"], msg["keys"])
        except Exception as e:  # noqa: BLE001 - EOF / reset / bad frame: this connection is done
            self._down(sock, e)

    def _down(self, sock, exc):
        with self.lock:
            if sock is not None and self.sock is not sock:
                return  # an older connection
            if self.sock is not None:
                try:
                    self.sock.close()
                except OSError:
                    pass
            self.sock = None
            if not self.plane._stop:
                self.down_since = self.down_since or time.monotonic()
                self.error = repr(exc)
            pend, self.pending = self.pending, {}
        err = ShardUnavailable(f"search shard {self.rank} unavailable: {exc!r}")
        for _, fail in pend.values():
            fail(err)

    def close(self):
        with self.lock:
            if self.sock is not None:
                try:
                    self.sock.shutdown(socket.SHUT_RDWR)
                    self.sock.close()
                except OSError:
                    pass
                self.sock = None


class SearchPlane:
    """One per rank: this rank's shard server + the client that routes searches to the owners.

    Single process: ``SearchPlane(index).start()``. Several ranks: ``listen()`` on every rank, one
    address exchange at startup (``start_world`` does it with a single gloo all-gather — the only
    collective the plane ever issues), ``connect(addrs)``, ``start()``."""

    def __init__(self, index, rank: int = 0, world: int = 1, device=None, stream=None, owner=None,
                 host: str = "127.0.0.1", port: int = 0, timeout_s: float = 30.0, max_rows: int = 1024,
                 retry_s: float = 1.0, connect_timeout_s: float = 2.0, send_timeout_s: float = 5.0):
        self.index, self.rank, self.world = index, rank, max(1, world)
        self.device = torch.device(device) if device is not None else getattr(index, "device", torch.device("cpu"))
        self.stream = stream  # None: a high-priority stream created by the scan worker
        self.owner = owner or (lambda d: owner_of(d, self.world))
        self.host, self.port = host, port
        self.timeout_s, self.max_rows = timeout_s, max_rows
        self.retry_s, self.connect_timeout_s, self.send_timeout_s = retry_s, connect_timeout_s, send_timeout_s
        self.addrs = None
        self.peers: dict[int, _Peer] = {}
        self.jobs: collections.deque = collections.deque()
        self.cv = threading.Condition()
        self.searches: dict[int, _Search] = {}
        self._ids = 0
        self._ids_lock = threading.Lock()
        self._stop = False
        self._threads: list[threading.Thread] = []
        self._listener = None
        self._conns: list = []
        self.error = ""
        self.stats = {"searches": 0, "local_parts": 0, "remote_parts": 0, "served_remote": 0, "scans": 0,
                      "rows": 0, "busy_s": 0.0, "failed": 0, "refused": 0, "expired": 0}
        self._queued_rows = 0

    # ------------------------------------------------------------------ lifecycle
    def listen(self) -> tuple:
        """Bind this rank's shard server; returns its (host, port)."""
        if self._listener is None:
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind((self.host, self.port))
            ls.listen(64)
            self._listener = ls
        return self._listener.getsockname()[:2]

    def connect(self, addrs) -> "SearchPlane":
        """Every rank's shard-server address, rank order (connections open lazily)."""
        self.addrs = [tuple(a) for a in addrs]
        if len(self.addrs) != self.world:
            raise ValueError(f"search plane: {len(self.addrs)} addresses for a world of {self.world}")
        self.peers = {r: _Peer(self, r, a) for r, a in enumerate(self.addrs) if r != self.rank}
        return self

    def start(self) -> "SearchPlane":
        if self.world > 1 and self.addrs is None:
            raise RuntimeError("search plane: connect(addrs) before start() when world > 1")
        for fn, name in ((self._scan_loop, "scan"), (self._housekeeping, "timer")):
            t = threading.Thread(target=fn, name=f"plane-{name}-{self.rank}", daemon=True)
            t.start()
            self._threads.append(t)
        if self._listener is not None:
            t = threading.Thread(target=self._accept_loop, name=f"plane-accept-{self.rank}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    @classmethod
    def start_world(cls, index, rank: int, world: int, group=None, **kw) -> "SearchPlane":
        """listen + exchange addresses over ``group`` (gloo; one all_gather_object at startup) +
        connect + start. Every rank of the world calls it."""
        plane = cls(index, rank, world, **kw)
        if world == 1:
            return plane.start()
        import torch.distributed as dist
        addr = plane.listen()
        addrs = [None] * world
        dist.all_gather_object(addrs, list(addr), group=group)
        return plane.connect(addrs).start()

    def stop(self, timeout: float = 10.0) -> None:
        self._stop = True
        with self.cv:
            self.cv.notify_all()
        if self._listener is not None:
            # shutdown first: close() alone neither wakes a thread blocked in accept() nor releases
            # the port while that call holds the socket (a restarted rank could not rebind)
            for fn in (lambda: self._listener.shutdown(socket.SHUT_RDWR), self._listener.close):
                try:
                    fn()
                except OSError:
                    pass
        for p in self.peers.values():
            p.close()
        for c in list(self._conns):
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass
        for t in self._threads:
            if t is not threading.current_thread():
                t.join(timeout)
        self._fail_all(RuntimeError("search plane stopped"))

    @property
    def healthy(self) -> bool:
        """This rank's shard server is serving (peers being down is reported by ``health``)."""
        return not self._stop and not self.error and all(t.is_alive() for t in self._threads)

    def health(self) -> dict:
        down = sorted(r for r, p in self.peers.items() if p.down_since is not None)
        return {"ok": self.healthy, "shards_down": down,
                "errors": {str(r): self.peers[r].error for r in down}}

    # ------------------------------------------------------------------ submit / route / merge
    def submit(self, vecs, k: int, min_sim: float, filters=None) -> cf.Future:
        """vecs [n, d]; filters: None (every document), or one document-id list per row (or one list
        for all rows). Future -> (scores fp32 [n, k], external ids int64 [n, k]), -inf / -1 padded."""
        vecs = np.ascontiguousarray(vecs, dtype=np.float32).reshape(-1, self.index.dim)
        n, k, thr = vecs.shape[0], int(k), float(min_sim)
        if filters is not None:
            if len(filters) == 1 and n != 1:
                filters = list(filters) * n
            if len(filters) != n:
                raise ValueError("search: one document filter per query row (or one for all rows)")
        fut: cf.Future = cf.Future()
        if self._stop or not self.healthy and self._threads:
            fut.set_exception(RuntimeError(f"search plane down: {self.error or 'stopped'}"))
            return fut
        # route: rank -> (rows, per-row filters restricted to that rank's documents)
        route: dict[int, tuple[list, list]] = {}
        for i in range(n):
            f = None if filters is None else filters[i]
            if f is None:
                for r in range(self.world):
                    rr = route.setdefault(r, ([], []))
                    rr[0].append(i)
                    rr[1].append(None)
                continue
            by: dict[int, list] = {}
            for d in f:
                by.setdefault(self.owner(str(d)), []).append(str(d))
            for r, ds in by.items():
                rr = route.setdefault(r, ([], []))
                rr[0].append(i)
                rr[1].append(ds)
        self.stats["searches"] += 1
        if not route:  # every row filters on nothing: nothing can match
            fut.set_result((np.full((n, k), -np.inf, np.float32), np.full((n, k), -1, np.int64)))
            return fut
        with self._ids_lock:
            self._ids += 1
            sid = self._ids
        srch = _Search(n, k, thr, route.keys(), fut, time.monotonic() + self.timeout_s)
        self.searches[sid] = srch
        for r, (rows, flt) in route.items():
            rows_a = np.asarray(rows, dtype=np.int64)

            def reply(s, g, r=r, rows_a=rows_a):
                self._part_done(sid, r, (rows_a, np.asarray(s, np.float32), np.asarray(g, np.int64)), None)

            def fail(exc, r=r):
                self._part_done(sid, r, None, exc)
            sub = vecs if len(rows) == n else vecs[rows_a]
            if r == self.rank:
                self.stats["local_parts"] += 1
                self._enqueue(_Job(sub, k, thr, flt, reply, fail))
            else:
                self.stats["remote_parts"] += 1
                self.peers[r].send(sid, {"id": sid, "vecs": sub, "k": k, "thr": thr, "filters": flt,
                                         "ttl": self.timeout_s}, reply, fail, deadline=srch.deadline)
        return fut

    def _part_done(self, sid: int, rank: int, part, exc):
        s = self.searches.get(sid)
        if s is None:
            return
        with s.lock:
            if s.fut.done() or rank not in s.ranks:
                return
            s.ranks.discard(rank)
            if exc is not None:
                self.searches.pop(sid, None)
                self.stats["failed"] += 1
                s.fut.set_exception(exc)
                return
            s.parts[rank] = part
            if s.ranks:
                return
            self.searches.pop(sid, None)
        try:
            s.fut.set_result(merge_host(s.parts, s.n, s.k, self.world, s.thr))
        except Exception as e:  # noqa: BLE001
            s.fut.set_exception(e)

    def _housekeeping(self):
        """Fail searches whose parts did not come back within ``timeout_s`` (a hung shard), naming
        the shards still pending."""
        while not self._stop:
            time.sleep(0.1)
            now = time.monotonic()
            for sid, s in list(self.searches.items()):
                if now > s.deadline:
                    pend = sorted(s.ranks)
                    for r in pend:
                        self._part_done(sid, r, None, TimeoutError(
                            f"search shards {pend} did not answer within {self.timeout_s:.0f} s"))
                        peer = self.peers.get(r)
                        if peer is not None:  # a hung peer never replies: drop the callbacks (and rows)
                            with peer.lock:
                                peer.pending.pop(sid, None)

    def _fail_all(self, exc):
        for sid, s in list(self.searches.items()):
            for r in list(s.ranks):
                self._part_done(sid, r, None, exc)
        with self.cv:
            jobs, self.jobs = list(self.jobs), collections.deque()
            self._queued_rows = 0
        for j in jobs:
            j.fail(exc)

    # ------------------------------------------------------------------ shard server
    def _accept_loop(self):
        while not self._stop:
            try:
                c, _ = self._listener.accept()
            except OSError:
                return
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._conns.append(c)
            threading.Thread(target=self._serve_conn, args=(c,), name=f"plane-conn-{self.rank}", daemon=True).start()

    def _serve_conn(self, c):
        # replies leave through this connection's own writer thread: the scan worker only queues
        # them, so a requester that stops reading (its receive buffer full) blocks its own writer,
        # never the shard's scans for everyone else; past _REPLY_BACKLOG queued replies the
        # connection is dropped (that requester fails its own pending parts)
        outq: queue.Queue = queue.Queue()
        dead = threading.Event()

        def writer():
            while True:
                obj = outq.get()
                if obj is None or dead.is_set():
                    return
                try:
                    _send_frame(c, obj)
                except OSError:
                    dead.set()
                    _close(c)
                    return

        def send(obj):
            if dead.is_set():
                return
            if outq.qsize() >= _REPLY_BACKLOG:
                dead.set()
                _close(c)
                return
            outq.put(obj)
        threading.Thread(target=writer, name=f"plane-reply-{self.rank}", daemon=True).start()
        try:
            while not self._stop:
                msg = _recv_frame(c)
                rid = msg.get("id")
                try:
                    vecs = np.ascontiguousarray(msg["vecs"], dtype=np.float32).reshape(-1, self.index.dim)
                    flt = msg.get("filters")
                    if flt is not None and len(flt) != vecs.shape[0]:
                        raise ValueError("one filter per row")
                    k = int(msg["k"])
                    if not 0 < k <= 1024:
                        raise ValueError(f"bad k {k}")
                except Exception as e:  # noqa: BLE001 - a malformed request fails alone
                    send({"id": rid, "error": f"bad request: {e}"})
                    continue
                self.stats["served_remote"] += 1
                ttl = msg.get("ttl")
                self._enqueue(_Job(vecs, k, float(msg["thr"]), flt,
                                   lambda s, g, rid=rid: send({"id": rid, "scores": s, "keys": g}),
                                   lambda e, rid=rid: send({"id": rid, "error": repr(e)}),
                                   None if ttl is None else time.monotonic() + float(ttl)))
        except Exception:  # noqa: BLE001 - EOF / reset: the requester's side handles it
            pass
        finally:
            dead.set()
            outq.put(None)
            _close(c)
            try:
                self._conns.remove(c)
            except ValueError:
                pass

    def _enqueue(self, job: _Job):
        """Queue a part for the scan worker; a shard already holding _QUEUED_ROWS_MAX query rows
        (its scan worker stalled: a GPU hang, a long IVF train) refuses it instead of growing."""
        with self.cv:
            if self._queued_rows + job.vecs.shape[0] > _QUEUED_ROWS_MAX:
                over = True
            else:
                over = False
                self.jobs.append(job)
                self._queued_rows += job.vecs.shape[0]
                self.cv.notify()
        if over:
            self.stats["refused"] += 1
            job.fail(ShardUnavailable(f"search shard {self.rank} overloaded ({_QUEUED_ROWS_MAX} rows queued)"))

    def _take(self) -> list[_Job]:
        out, n, expired = [], 0, []
        with self.cv:
            while not self.jobs and not self._stop:
                self.cv.wait(0.5)
            now = time.monotonic()
            while self.jobs and (not out or n + self.jobs[0].vecs.shape[0] <= self.max_rows):
                j = self.jobs.popleft()
                self._queued_rows -= j.vecs.shape[0]
                if j.deadline is not None and now > j.deadline:
                    expired.append(j)  # its requester has given up: do not scan it
                    continue
                out.append(j)
                n += j.vecs.shape[0]
        for j in expired:
            self.stats["expired"] += 1
            j.fail(TimeoutError("search part expired in the shard's queue"))
        return out

    def _scan_loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        while not self._stop:
            take = self._take()
            if not take:
                continue
            try:
                self._scan(take)
            except Exception as e:  # noqa: BLE001 - fail this batch's parts, keep serving
                for j in take:
                    j.fail(e)

    def _scan(self, take: list[_Job]):
        """ONE fused scan for every queued part (local and remote) on this rank's shard."""
        t0 = time.perf_counter()
        idx, dev = self.index, self.index.device
        K = max(j.k for j in take)
        thr = min(j.thr for j in take)
        Q = np.concatenate([j.vecs for j in take])
        filters = [f for j in take for f in (j.filters if j.filters is not None else [None] * j.vecs.shape[0])]
        nofilter = all(f is None for f in filters)
        stream_ctx = torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()
        ws_ctx = _nullctx()
        if dev.type == "cuda":
            # the scan kernels' scratch must not be the GPU thread's: its decode graph captured that
            # workspace's pointer and runs concurrently with this thread (ops/kernels.py workspace_role)
            from ..ops.kernels import workspace_role
            ws_ctx = workspace_role("search")
        with stream_ctx, ws_ctx:
            # search_ids orders this stream after the shard's last committed write (index/flat.py)
            s, g = idx.search_ids(torch.from_numpy(Q).to(dev), K, thr, None if nofilter else filters)
            s, g = s.float().cpu().numpy(), g.cpu().numpy()
        o = 0
        for j in take:
            m = j.vecs.shape[0]
            sc, ky = s[o:o + m, :j.k].copy(), g[o:o + m, :j.k].copy()
            drop = ~(sc >= j.thr)
            sc[drop], ky[drop] = -np.inf, -1
            j.reply(sc, ky)
            o += m
        self.stats["scans"] += 1
        self.stats["rows"] += len(Q)
        self.stats["busy_s"] += time.perf_counter() - t0


def _close(sock):
    for fn in (lambda: sock.shutdown(socket.SHUT_RDWR), sock.close):
        try:
            fn()
        except OSError:
            pass


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
