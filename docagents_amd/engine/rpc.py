"""Engine RPC: length-prefixed msgpack frames over TCP (or a unix socket).

Frame: 4-byte big-endian length + msgpack map. Request ``{"id", "method", "args", "trace"}``,
response ``{"id", "result"}`` or ``{"id", "error"}``. numpy arrays travel as msgpack ext type 1
(``dtype|shape|raw bytes``), so 768-d vectors cost 3 KB, not a JSON float list (the reference
serialised 3072 floats as decimal text per row, internal/store/postgres.go:321-330).

The server side lives in ``engine/server.py``; ``EngineClient`` is used by the agents (it
pipelines concurrent calls over one connection, so their requests reach the micro-batcher
together).
"""
from __future__ import annotations

import asyncio
import itertools
import struct
import time

import msgpack
import numpy as np

_ND = 1


def _default(o):
    if isinstance(o, np.ndarray):
        hdr = f"{o.dtype.str}|{','.join(map(str, o.shape))}".encode()
        return msgpack.ExtType(_ND, struct.pack(">H", len(hdr)) + hdr + np.ascontiguousarray(o).tobytes())
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    raise TypeError(f"cannot serialise {type(o)}")


def _ext_hook(code, data):
    if code == _ND:
        n = struct.unpack(">H", data[:2])[0]
        dt, shape = data[2:2 + n].decode().split("|")
        shp = tuple(int(x) for x in shape.split(",") if x)
        return np.frombuffer(data[2 + n:], dtype=np.dtype(dt)).reshape(shp).copy()
    return msgpack.ExtType(code, data)


def dumps(obj) -> bytes:
    """msgpack with numpy arrays as ext type 1 (the engine's data-plane payload encoding)."""
    return msgpack.packb(obj, default=_default, use_bin_type=True)


def loads(b: bytes):
    return msgpack.unpackb(b, ext_hook=_ext_hook, raw=False, strict_map_key=False)


def pack(obj) -> bytes:
    b = msgpack.packb(obj, default=_default, use_bin_type=True)
    return struct.pack(">I", len(b)) + b


def unpack(b: bytes):
    return msgpack.unpackb(b, ext_hook=_ext_hook, raw=False, strict_map_key=False)


async def read_frame(reader: asyncio.StreamReader):
    hdr = await reader.readexactly(4)
    n = struct.unpack(">I", hdr)[0]
    return unpack(await reader.readexactly(n))


class RPCError(RuntimeError):
    pass


def parse_url(url: str):
    """tcp://host:port | unix:///path | host:port"""
    if url.startswith("unix://"):
        return ("unix", url[len("unix://"):])
    if url.startswith("tcp://"):
        url = url[len("tcp://"):]
    host, _, port = url.rpartition(":")
    return ("tcp", (host or "127.0.0.1", int(port)))


class EngineClient:
    def __init__(self, url: str, timeout: float = 120.0):
        self.url, self.timeout = url, timeout
        self.reader = self.writer = None
        self.pending: dict[int, asyncio.Future] = {}
        self.ids = itertools.count(1)
        self.reader_task = None
        self.lock = asyncio.Lock()

    async def connect(self, retries: int = 1, delay: float = 0.5):
        kind, addr = parse_url(self.url)
        last = None
        for _ in range(max(1, retries)):
            try:
                if kind == "unix":
                    self.reader, self.writer = await asyncio.open_unix_connection(addr)
                else:
                    self.reader, self.writer = await asyncio.open_connection(*addr)
                break
            except OSError as e:
                last = e
                await asyncio.sleep(delay)
        else:
            raise ConnectionError(f"engine unreachable at {self.url}: {last}")
        self.reader_task = asyncio.ensure_future(self._read_loop())
        return self

    async def _read_loop(self):
        try:
            while True:
                msg = await read_frame(self.reader)
                fut = self.pending.pop(msg.get("id"), None)
                if fut is not None and not fut.done():
                    if "error" in msg:
                        fut.set_exception(RPCError(msg["error"]))
                    else:
                        fut.set_result(msg.get("result"))
        except (asyncio.IncompleteReadError, ConnectionError, OSError) as e:
            # the next call reconnects (a restarted engine is picked up; a dead one fails fast)
            w, self.writer = self.writer, None
            if w is not None:
                w.close()
            for f in self.pending.values():
                if not f.done():
                    f.set_exception(ConnectionError(f"engine connection lost: {e}"))
            self.pending.clear()

    async def call(self, method: str, trace: str = "", **args):
        if self.writer is None:
            await self.connect()
        rid = next(self.ids)
        fut = asyncio.get_running_loop().create_future()
        self.pending[rid] = fut
        try:
            async with self.lock:
                if self.writer is None:
                    raise ConnectionError(f"engine connection to {self.url} lost")
                self.writer.write(pack({"id": rid, "method": method, "args": args, "trace": trace}))
                await self.writer.drain()
        except (ConnectionError, OSError) as e:
            self.pending.pop(rid, None)
            raise ConnectionError(f"engine at {self.url}: {e}") from e
        try:
            return await asyncio.wait_for(fut, self.timeout)
        finally:
            self.pending.pop(rid, None)

    async def close(self):
        if self.reader_task:
            self.reader_task.cancel()
        if self.writer:
            self.writer.close()
            self.writer = None


def _owner(doc_id: str, world: int) -> int:
    from .server import owner_of
    return owner_of(doc_id, world)


class EngineCluster:
    """Client of a replicated engine (``TP_SIZE`` < world): one ``EngineClient`` per replica.

    ``connect`` reaches the configured URL (replica 0), asks it for the topology and connects to
    every replica. ``call`` keeps the single-client interface:
      * index mutations (``index_add``, ``embed_index``, ``index_remove``) go to the replica that
        owns the document's shard (rank hash(doc_id) % world — the engine rejects misrouted ones);
      * ``index_docs`` / ``stats`` / ``checkpoint`` / ``ping`` fan out to every replica and merge;
      * everything else (embed, embed_search, search, answer, summarize) goes to the replica with
        the fewest calls in flight — the reference's queue-group load balancing
        (internal/queue/nats.go:40-51) for the GPU engine. These calls are idempotent (no engine
        state changes), so a replica that is unreachable (or reports itself unhealthy) is skipped
        for ``dead_s`` and the call is retried on the next live replica: replicas fail
        independently, as the reference's queue-group workers do. A client-side timeout is not a
        dead replica: cheap calls (embed / search) are re-asked of another replica, generations
        (answer / summarize) fail — nothing cancels them server-side, so a retry would double the work;
      * ``health`` fans out: healthy only if every replica is, with the dead ones named.
    ``stats`` has one shape for any replica count: ``{"replicas": [per-replica stats]}``."""

    ROUTED = ("index_add", "embed_index", "index_remove")
    FANOUT = ("index_docs", "stats", "checkpoint", "ping")
    RETRYABLE = ("embed", "embed_search", "search", "answer", "summarize")

    def __init__(self, url: str, timeout: float = 120.0, dead_s: float = 2.0):
        self.url, self.timeout, self.dead_s = url, timeout, dead_s
        self.clients: list[EngineClient] = []
        self.inflight: list[int] = []
        self.dead_until: list[float] = []
        self.topology: dict = {"replicas": 1, "tp": 1, "world": 1}
        self._rr = 0

    async def connect(self, retries: int = 1, delay: float = 0.5):
        first = await EngineClient(self.url, self.timeout).connect(retries, delay)
        try:
            topo = await first.call("topology")
        except RPCError:  # an engine without the topology RPC: a single replica
            topo = {"replicas": 1, "tp": 1, "world": 1, "urls": [self.url]}
        self.topology = topo
        self.clients = [first]
        kind, addr = parse_url(self.url)
        for r in range(1, int(topo.get("replicas", 1))):
            u = topo["urls"][r]
            if kind == "tcp":  # reach the other replicas on the host this client used for replica 0
                _, (_, port) = parse_url(u)
                u = f"tcp://{addr[0]}:{port}"
            self.clients.append(await EngineClient(u, self.timeout).connect(retries, delay))
        self.inflight = [0] * len(self.clients)
        self.dead_until = [0.0] * len(self.clients)
        return self

    @property
    def replicas(self) -> int:
        return len(self.clients)

    def replica_of(self, doc_id: str) -> int:
        return _owner(str(doc_id), int(self.topology.get("world", 1))) // int(self.topology.get("tp", 1))

    def _pick(self, exclude=()) -> int:
        n = len(self.clients)
        now = time.monotonic()
        cand = [i for i in range(n) if i not in exclude] or list(range(n))
        best = min(cand, key=lambda i: (self.dead_until[i] > now, self.inflight[i], (i - self._rr) % n))
        self._rr = (best + 1) % n
        return best

    CHEAP = ("embed", "embed_search", "search")  # a timed-out one may be re-asked of another replica

    @staticmethod
    def _replica_down(e: BaseException) -> bool:
        """A failure of the replica itself (not of the request): connection lost / refused, or the
        engine's watchdog reporting it unhealthy. NOT a client-side timeout: a busy replica is
        alive (marking it dead would steer load off live replicas and, for generations, re-run the
        same work elsewhere while the first replica still computes it — a retry storm)."""
        if isinstance(e, (asyncio.TimeoutError, TimeoutError)):
            return False
        return isinstance(e, (ConnectionError, OSError)) or (isinstance(e, RPCError) and "engine unhealthy" in str(e))

    async def _on(self, i: int, method: str, trace: str, args: dict):
        self.inflight[i] += 1
        try:
            return await self.clients[i].call(method, trace=trace, **args)
        finally:
            self.inflight[i] -= 1

    async def call(self, method: str, trace: str = "", **args):
        if self.writer_missing():
            await self.connect()
        if method == "health":
            return await self._health(trace)
        if method == "stats":
            return {"replicas": await asyncio.gather(*[self._on(i, method, trace, args)
                                                       for i in range(len(self.clients))])}
        if len(self.clients) == 1:
            return await self._on(0, method, trace, args)
        if method in self.ROUTED:
            doc = args["doc_id"] if "doc_id" in args else args["items"][0][0]
            return await self._on(self.replica_of(doc), method, trace, args)
        if method in self.FANOUT:
            parts = await asyncio.gather(*[self._on(i, method, trace, args) for i in range(len(self.clients))])
            if method == "index_docs":
                merged: dict = {}
                for p in parts:
                    for d, n in p.items():
                        merged[d] = merged.get(d, 0) + n
                return merged
            if method == "checkpoint":
                return sum(parts)
            if method == "ping":
                return [r for p in parts for r in p]
            return {"replicas": parts}
        if method not in self.RETRYABLE:
            return await self._on(self._pick(), method, trace, args)
        tried: list[int] = []
        while True:
            i = self._pick(tried)
            tried.append(i)
            try:
                return await self._on(i, method, trace, args)
            except Exception as e:  # noqa: BLE001
                if len(tried) >= len(self.clients):
                    raise
                if self._replica_down(e):
                    self.dead_until[i] = time.monotonic() + self.dead_s
                elif not (isinstance(e, (asyncio.TimeoutError, TimeoutError)) and method in self.CHEAP):
                    raise  # a request error, or a timed-out generation: fail the call, retry nothing

    async def _health(self, trace: str = ""):
        async def one(i):
            try:
                return await asyncio.wait_for(self.clients[i].call("health", trace=trace), min(self.timeout, 10.0))
            except Exception as e:  # noqa: BLE001 - a dead replica is a health result, not an error
                return {"ok": False, "replica": i, "error": f"{type(e).__name__}: {e}"}
        parts = await asyncio.gather(*[one(i) for i in range(len(self.clients))])
        if len(parts) == 1:
            return parts[0]
        dead = [i for i, p in enumerate(parts) if "error" in p]
        down = sorted({r for p in parts for r in p.get("shards_down", [])})
        return {"ok": all(bool(p.get("ok")) for p in parts), "replicas": parts, "dead_replicas": dead,
                "shards_down": down}

    def writer_missing(self) -> bool:
        return not self.clients

    async def close(self):
        for c in self.clients:
            await c.close()
        self.clients = []
