"""Keep-alive HTTP/1.1 client for the gateway -> query proxy (cmd/gateway/main.go:180-207).

The reference forwards ``POST /api/query`` with Go's pooled ``http.Client``. A general-purpose
Python client (httpx) adds ~2.5 ms per hop on the cache-hit path, which is otherwise ~1 ms end to
end, so the gateway uses this small pooled client instead: plain ``http://`` only, one request in
flight per pooled connection, Content-Length or chunked response bodies, a stale pooled
connection is retried once on a fresh one. Anything else (``https://``) goes through httpx.
"""
from __future__ import annotations

import asyncio
from urllib.parse import urlsplit


class ProxyError(RuntimeError):
    pass


class PooledHTTPClient:
    def __init__(self, timeout: float = 60.0, max_idle: int = 128):
        self.timeout, self.max_idle = timeout, max_idle
        self._idle: dict[tuple[str, int], list] = {}
        self._fallback = None

    async def post(self, url: str, body: bytes, headers: dict[str, str]) -> tuple[int, bytes]:
        u = urlsplit(url)
        if u.scheme != "http":
            return await self._post_httpx(url, body, headers)
        host, port = u.hostname or "127.0.0.1", u.port or 80
        path = (u.path or "/") + (f"?{u.query}" if u.query else "")
        head = [f"POST {path} HTTP/1.1", f"Host: {host}:{port}", f"Content-Length: {len(body)}"]
        head += [f"{k}: {v}" for k, v in headers.items()]
        req = ("\r\n".join(head) + "\r\n\r\n").encode("latin-1") + body
        return await asyncio.wait_for(self._roundtrip((host, port), req), self.timeout)

    async def _roundtrip(self, key, req: bytes) -> tuple[int, bytes]:
        pool = self._idle.setdefault(key, [])
        while pool:
            r, w = pool.pop()
            if w.is_closing() or r.at_eof():
                w.close()
                continue
            try:
                return await self._exchange(key, r, w, req)
            except (ConnectionError, asyncio.IncompleteReadError, ProxyError):
                w.close()  # the server closed an idle connection: retry on a fresh one
                break
        r, w = await asyncio.open_connection(*key)
        try:
            return await self._exchange(key, r, w, req)
        except BaseException:
            w.close()
            raise

    async def _exchange(self, key, r, w, req: bytes) -> tuple[int, bytes]:
        w.write(req)
        await w.drain()
        raw = await r.readuntil(b"\r\n\r\n")
        lines = raw.decode("latin-1").split("\r\n")
        parts = lines[0].split(" ", 2)
        if len(parts) < 2 or not parts[0].startswith("HTTP/1."):
            raise ProxyError(f"bad status line {lines[0]!r}")
        status = int(parts[1])
        hdr = {}
        for ln in lines[1:]:
            if ":" in ln:
                k, v = ln.split(":", 1)
                hdr[k.strip().lower()] = v.strip()
        if "content-length" in hdr:
            body = await r.readexactly(int(hdr["content-length"]))
        elif "chunked" in hdr.get("transfer-encoding", "").lower():
            chunks = []
            while True:
                size = int((await r.readuntil(b"\r\n")).split(b";")[0].strip(), 16)
                if size == 0:
                    await r.readuntil(b"\r\n")  # no trailers from our services
                    break
                chunks.append(await r.readexactly(size))
                await r.readexactly(2)
            body = b"".join(chunks)
        else:  # body delimited by connection close
            body = await r.read()
            hdr["connection"] = "close"
        if hdr.get("connection", "").lower() == "close" or parts[0] == "HTTP/1.0":
            w.close()
        else:
            pool = self._idle.setdefault(key, [])
            if len(pool) < self.max_idle:
                pool.append((r, w))
            else:
                w.close()
        return status, body

    async def _post_httpx(self, url, body, headers):
        import httpx
        if self._fallback is None:
            self._fallback = httpx.AsyncClient(timeout=self.timeout)
        resp = await self._fallback.post(url, content=body, headers=headers)
        return resp.status_code, resp.content

    async def aclose(self):
        for pool in self._idle.values():
            for _, w in pool:
                w.close()
        self._idle.clear()
        if self._fallback is not None:
            await self._fallback.aclose()
