"""Query-result and question-embedding caches (internal/cache/*).

Contract (cache.go:13-33): get/set query result, get/set embedding (keyed by the RAW question
text — reference quirk), invalidate, close. ``get_*`` returns None on a miss.

Providers:
  * ``MemoryCache`` — in-process TTL dict (tests / single-process deployments).
  * ``NoOpCache``   — always miss, always succeed (cache/noop.go; the fallback when the KV server is
                      unreachable, internal/app/deps.go:129-134).
  * ``KVCache``     — RESP client for the in-repo native KV server (``docagents_amd/native/kvserver``)
                      or a real Redis: keys ``query:<sha256>`` / ``embed:<sha256>``, JSON values with
                      the reference's field names (``Answer``/``Confidence``/``Sources``), TTL via EX.
"""
from __future__ import annotations

import asyncio
import collections
import json
import time
from dataclasses import dataclass, field

from ..utils import faults
from .keys import EMBED_PREFIX, QUERY_PREFIX, generate_embedding_key


@dataclass
class Source:
    chunk_id: str
    score: float
    preview: str

    def to_json(self):
        from ..api.gojson import F32, Struct
        return Struct(chunk_id=self.chunk_id, score=F32(self.score), preview=self.preview)


@dataclass
class QueryResult:
    answer: str
    confidence: float
    sources: list[Source] = field(default_factory=list)

    def encode(self) -> bytes:
        from ..api.gojson import F32, Struct, dumps_compact
        return dumps_compact(Struct(Answer=self.answer, Confidence=F32(self.confidence),
                                    Sources=[s.to_json() for s in self.sources] if self.sources is not None else None)
                             ).encode()

    @classmethod
    def decode(cls, data: bytes) -> "QueryResult":
        d = json.loads(data)
        src = [Source(s.get("chunk_id", ""), float(s.get("score", 0.0)), s.get("preview", ""))
               for s in (d.get("Sources") or [])]
        return cls(d.get("Answer", ""), float(d.get("Confidence", 0.0)), src)


class NoOpCache:
    async def get_query_result(self, key: str):
        return None

    async def set_query_result(self, key: str, result: QueryResult, ttl: float):
        return None

    async def get_embedding(self, text: str):
        return None

    async def set_embedding(self, text: str, vector, ttl: float):
        return None

    async def invalidate_document(self, doc_id: str):
        return None

    async def close(self):
        return None


class MemoryCache:
    def __init__(self, clock=time.monotonic):
        self.d: dict[str, tuple[float, bytes]] = {}
        self.clock = clock
        self.hits = self.misses = 0

    def _get(self, key):
        faults.maybe_fail("cache.get")
        v = self.d.get(key)
        if v is None:
            self.misses += 1
            return None
        exp, data = v
        if exp and self.clock() >= exp:
            del self.d[key]
            self.misses += 1
            return None
        self.hits += 1
        return data

    def _set(self, key, data: bytes, ttl: float):
        faults.maybe_fail("cache.set")
        self.d[key] = ((self.clock() + ttl) if ttl and ttl > 0 else 0.0, data)

    async def get_query_result(self, key: str):
        data = self._get(QUERY_PREFIX + key)
        return None if data is None else QueryResult.decode(data)

    async def set_query_result(self, key: str, result: QueryResult, ttl: float):
        self._set(QUERY_PREFIX + key, result.encode(), ttl)

    async def get_embedding(self, text: str):
        data = self._get(EMBED_PREFIX + generate_embedding_key(text))
        return None if data is None else json.loads(data)

    async def set_embedding(self, text: str, vector, ttl: float):
        self._set(EMBED_PREFIX + generate_embedding_key(text), json.dumps([float(x) for x in vector]).encode(), ttl)

    async def invalidate_document(self, doc_id: str):
        # reference behaviour (redis.go:110-138): drops EVERY cached query result
        for k in [k for k in self.d if k.startswith(QUERY_PREFIX)]:
            del self.d[k]

    async def close(self):
        self.d.clear()


class RespError(RuntimeError):
    pass


def _resp_cmd(*parts) -> bytes:
    out = [f"*{len(parts)}\r\n".encode()]
    for p in parts:
        b = p if isinstance(p, bytes) else str(p).encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


class KVCache:
    """Minimal asyncio RESP client (GET/SET EX/DEL/SCAN/PING/AUTH), pipelined: a command is written
    as soon as it is issued and its reply matched in FIFO order by one reader task (RESP answers in
    request order), so concurrent requests share the connection without waiting for each other's
    round trips — the reference's go-redis pools connections for the same reason. A command that
    times out keeps its place in the FIFO (its late reply is read and dropped). A lost connection
    fails the commands in flight; the next command reconnects (go-redis's behaviour), at most one
    attempt per ``RECONNECT_S`` so a dead server costs the callers a fast error, not a connect
    timeout each."""

    RECONNECT_S = 1.0

    def __init__(self, addr: str = "localhost:6379", password: str = "", timeout: float = 5.0):
        host, _, port = addr.rpartition(":")
        self.host, self.port = host or "localhost", int(port or 6379)
        self.password, self.timeout = password, timeout
        self.reader = self.writer = None
        self.lock = asyncio.Lock()  # write order == FIFO order
        self._fifo: collections.deque = collections.deque()
        self._reader_task = None
        self._last_attempt = 0.0
        self.reconnects = 0

    async def connect(self):
        self.reader, self.writer = await asyncio.wait_for(asyncio.open_connection(self.host, self.port), self.timeout)
        self._reader_task = asyncio.ensure_future(self._read_loop(self.reader))
        if self.password:
            await self._cmd("AUTH", self.password)
        r = await self._cmd("PING")
        if r not in (b"PONG", "PONG"):
            raise RespError(f"unexpected PING reply {r!r}")
        return self

    async def _read(self, reader):
        line = await reader.readline()
        if not line:
            raise ConnectionError("kv connection closed")
        t, rest = line[:1], line[1:-2]
        if t == b"+":
            return rest
        if t == b"-":
            return RespError(rest.decode())  # this command's error, not the connection's
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            data = await reader.readexactly(n + 2)
            return data[:-2]
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [await self._read(reader) for _ in range(n)]
        raise ConnectionError(f"bad RESP type {t!r}")

    async def _read_loop(self, reader):
        try:
            while True:
                v = await self._read(reader)
                fut = self._fifo.popleft() if self._fifo else None
                if fut is None or fut.done():
                    continue  # timed out / cancelled: its reply is dropped, the order kept
                if isinstance(v, RespError):
                    fut.set_exception(v)
                else:
                    fut.set_result(v)
        except (ConnectionError, asyncio.IncompleteReadError, OSError, ValueError) as e:
            err = e if isinstance(e, ConnectionError) else ConnectionError(f"kv connection lost: {e!r}")
            w, self.writer = self.writer, None
            if w is not None:
                w.close()
            while self._fifo:
                f = self._fifo.popleft()
                if not f.done():
                    f.set_exception(err)

    async def _reconnect_locked(self):
        """(self.lock held) open a new connection after a loss; AUTH goes first in its FIFO."""
        now = time.monotonic()
        if self._last_attempt and now - self._last_attempt < self.RECONNECT_S:
            raise ConnectionError("kv cache not connected (reconnect backoff)")
        self._last_attempt = now
        reader, writer = await asyncio.wait_for(asyncio.open_connection(self.host, self.port), self.timeout)
        self.reader, self.writer = reader, writer
        self._reader_task = asyncio.ensure_future(self._read_loop(reader))
        self.reconnects += 1
        if self.password:
            auth = asyncio.get_running_loop().create_future()
            auth.add_done_callback(lambda f: f.cancelled() or f.exception())  # a bad AUTH fails the next command
            self._fifo.append(auth)
            writer.write(_resp_cmd("AUTH", self.password))

    async def _cmd(self, *parts):
        fut = asyncio.get_running_loop().create_future()
        async with self.lock:
            if self.writer is None:
                if self.reader is None:
                    raise ConnectionError("not connected")
                await self._reconnect_locked()
            self._fifo.append(fut)
            self.writer.write(_resp_cmd(*parts))
        w = self.writer
        if w is not None:
            await w.drain()
        return await asyncio.wait_for(fut, self.timeout)

    async def get_query_result(self, key: str):
        faults.maybe_fail("cache.get")
        data = await self._cmd("GET", QUERY_PREFIX + key)
        return None if data is None else QueryResult.decode(data)

    async def set_query_result(self, key: str, result: QueryResult, ttl: float):
        faults.maybe_fail("cache.set")
        await self._cmd("SET", QUERY_PREFIX + key, result.encode(), "EX", max(1, int(ttl)))

    async def get_embedding(self, text: str):
        faults.maybe_fail("cache.get")
        data = await self._cmd("GET", EMBED_PREFIX + generate_embedding_key(text))
        return None if data is None else json.loads(data)

    async def set_embedding(self, text: str, vector, ttl: float):
        faults.maybe_fail("cache.set")
        await self._cmd("SET", EMBED_PREFIX + generate_embedding_key(text),
                        json.dumps([float(x) for x in vector]), "EX", max(1, int(ttl)))

    async def invalidate_document(self, doc_id: str):
        cursor = b"0"
        keys = []
        while True:
            cursor, batch = await self._cmd("SCAN", cursor, "MATCH", QUERY_PREFIX + "*", "COUNT", 1000)
            keys.extend(batch)
            if cursor in (b"0", 0, "0"):
                break
        if keys:
            await self._cmd("DEL", *keys)

    async def close(self):
        if self._reader_task is not None:
            self._reader_task.cancel()
            self._reader_task = None
        if self.writer is not None:
            self.writer.close()
            try:
                await self.writer.wait_closed()
            except Exception:  # noqa: BLE001
                pass
            self.writer = None
        self.reader = None  # closed on purpose: no reconnect
