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
        async with self.lock:
            self.writer.write(pack({"id": rid, "method": method, "args": args, "trace": trace}))
            await self.writer.drain()
        return await asyncio.wait_for(fut, self.timeout)

    async def close(self):
        if self.reader_task:
            self.reader_task.cancel()
        if self.writer:
            self.writer.close()
            self.writer = None
