"""Minimal asyncio HTTP/1.1 server for the agents' ASGI apps (replaces uvicorn's pure-Python h11
stack on the request path; ``DA_HTTP_SERVER=uvicorn`` switches back).

The reference serves with Go's net/http (internal/httputil/httputil.go:25-34, cmd/*/main.go). With
uvicorn + h11 (httptools / uvloop are not installed) a cache-hit query costs ~1 ms of HTTP
parsing and task plumbing around a ~70 us handler; this server parses with bytes.split on an
``asyncio.Protocol``, runs one ASGI call per request (keep-alive, pipelined requests served in
order), and writes the response in one ``transport.write``.

Supported: Content-Length and chunked request bodies (<= ``max_body``), Content-Length or
streamed (chunked) responses, ``Connection: close``, HTTP/1.0. Not supported (not used by the
services): Expect: 100-continue (answered with 100 and then served), upgrades, trailers.
"""
from __future__ import annotations

import asyncio
import os

_REASONS = {200: b"OK", 201: b"Created", 202: b"Accepted", 204: b"No Content", 400: b"Bad Request", 404: b"Not Found",
            405: b"Method Not Allowed", 411: b"Length Required", 413: b"Payload Too Large",
            500: b"Internal Server Error", 503: b"Service Unavailable", 504: b"Gateway Timeout"}


class _Conn(asyncio.Protocol):
    def __init__(self, app, max_body: int, server_addr):
        self.app, self.max_body, self.server_addr = app, max_body, server_addr
        self.buf = bytearray()
        self.transport = None
        self.queue: asyncio.Queue = asyncio.Queue()
        self.task = None
        self.closed = False

    # ---------------------------------------------------------------- asyncio.Protocol
    def connection_made(self, transport):
        self.transport = transport
        self.peer = transport.get_extra_info("peername") or ("", 0)
        self.task = asyncio.get_running_loop().create_task(self._serve())

    def data_received(self, data):
        self.buf += data
        self.queue.put_nowait(None)

    def eof_received(self):
        self.closed = True
        self.queue.put_nowait(None)
        return False

    def connection_lost(self, exc):
        self.closed = True
        self.queue.put_nowait(None)

    # ---------------------------------------------------------------- request loop
    async def _need(self, pred):
        while not pred():
            if self.closed:
                return False
            await self.queue.get()
        return True

    async def _serve(self):
        try:
            while True:
                if not await self._need(lambda: b"\r\n\r\n" in self.buf):
                    return
                end = self.buf.index(b"\r\n\r\n")
                head = bytes(self.buf[:end])
                del self.buf[:end + 4]
                lines = head.split(b"\r\n")
                try:
                    method, target, version = lines[0].split(b" ", 2)
                except ValueError:
                    return self._simple(400, close=True)
                headers = []
                clen, chunked, keep = None, False, version == b"HTTP/1.1"
                for ln in lines[1:]:
                    k, _, v = ln.partition(b":")
                    k, v = k.strip().lower(), v.strip()
                    headers.append((k, v))
                    if k == b"content-length":
                        clen = int(v)
                    elif k == b"transfer-encoding" and b"chunked" in v.lower():
                        chunked = True
                    elif k == b"connection":
                        lv = v.lower()
                        keep = b"close" not in lv and (keep or b"keep-alive" in lv)
                    elif k == b"expect" and v.lower() == b"100-continue":
                        self.transport.write(version + b" 100 Continue\r\n\r\n")
                if chunked:
                    body = await self._read_chunked()
                    if body is None:
                        return
                else:
                    n = clen or 0
                    if n > self.max_body:
                        return self._simple(413, close=True)
                    if not await self._need(lambda: len(self.buf) >= n):
                        return
                    body = bytes(self.buf[:n])
                    del self.buf[:n]
                path, _, query = target.partition(b"?")
                scope = {
                    "type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"},
                    "http_version": version[5:].decode("latin-1"), "method": method.decode("latin-1"),
                    "scheme": "http", "path": _unquote(path), "raw_path": path, "query_string": query,
                    "root_path": "", "headers": headers, "client": self.peer[:2], "server": self.server_addr,
                }
                if not await self._call(scope, body, keep):
                    return
                if not keep:
                    self.transport.close()
                    return
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:  # the loop only exits to end the connection
            if self.transport is not None and not self.transport.is_closing():
                self.transport.close()

    async def _read_chunked(self):
        chunks, total = [], 0
        while True:
            if not await self._need(lambda: b"\r\n" in self.buf):
                return None
            i = self.buf.index(b"\r\n")
            size = int(bytes(self.buf[:i]).split(b";")[0].strip() or b"0", 16)
            del self.buf[:i + 2]
            if size == 0:
                if not await self._need(lambda: b"\r\n" in self.buf):
                    return None
                del self.buf[:self.buf.index(b"\r\n") + 2]  # trailers ignored
                return b"".join(chunks)
            total += size
            if total > self.max_body:
                self._simple(413, close=True)
                return None
            if not await self._need(lambda: len(self.buf) >= size + 2):
                return None
            chunks.append(bytes(self.buf[:size]))
            del self.buf[:size + 2]

    async def _call(self, scope, body: bytes, keep: bool) -> bool:
        state = {"sent_body": False, "status": 200, "headers": [], "chunks": [], "streaming": False, "done": False}
        delivered = False

        async def receive():
            nonlocal delivered
            if not delivered:
                delivered = True
                return {"type": "http.request", "body": body, "more_body": False}
            while not self.closed and not state["done"]:
                await asyncio.sleep(0.05)
            return {"type": "http.disconnect"}

        async def send(msg):
            t = msg["type"]
            if t == "http.response.start":
                state["status"] = msg["status"]
                state["headers"] = list(msg.get("headers", []))
            elif t == "http.response.body":
                chunk = msg.get("body", b"")
                more = msg.get("more_body", False)
                if more and not state["streaming"]:
                    state["streaming"] = True
                    self._write_head(state["status"], state["headers"], None, keep)
                if state["streaming"]:
                    if chunk:
                        self.transport.write(b"%x\r\n%s\r\n" % (len(chunk), chunk))
                    if not more:
                        self.transport.write(b"0\r\n\r\n")
                        state["done"] = True
                else:
                    self._write_head(state["status"], state["headers"], chunk, keep)
                    state["done"] = True

        try:
            await self.app(scope, receive, send)
        except Exception:  # noqa: BLE001 - the agents' Middleware already maps errors to 500
            if not state["done"]:
                self._simple(500, close=True)
            return False
        if not state["done"]:
            self._simple(500, close=True)
            return False
        return True

    def _write_head(self, status: int, headers, body, keep: bool):
        out = [b"HTTP/1.1 %d %s" % (status, _REASONS.get(status, b"Status"))]
        has_len = False
        for k, v in headers:
            kl = k.lower()
            if kl == b"content-length":
                if body is None:
                    continue  # streamed: chunked framing instead
                has_len = True
            out.append(k + b": " + v)
        if body is None:
            out.append(b"transfer-encoding: chunked")
        elif not has_len:
            out.append(b"content-length: %d" % len(body))
        if not keep:
            out.append(b"connection: close")
        self.transport.write(b"\r\n".join(out) + b"\r\n\r\n" + (body or b""))

    def _simple(self, status: int, close: bool = False):
        msg = _REASONS.get(status, b"Error") + b"\n"
        self._write_head(status, [(b"content-type", b"text/plain; charset=utf-8")], msg, not close)
        if close:
            self.transport.close()


def _unquote(p: bytes) -> str:
    if b"%" not in p:
        return p.decode("latin-1")
    from urllib.parse import unquote_to_bytes
    return unquote_to_bytes(p).decode("utf-8", "replace")


async def serve(app, host: str, port: int, max_body: int | None = None):
    """Serve ``app`` until cancelled."""
    max_body = max_body or int(os.environ.get("DA_HTTP_MAX_BODY", str(64 << 20)))
    loop = asyncio.get_running_loop()
    srv = await loop.create_server(lambda: _Conn(app, max_body, (host, port)), host, port, reuse_address=True,
                                   backlog=1024)
    async with srv:
        await srv.serve_forever()
