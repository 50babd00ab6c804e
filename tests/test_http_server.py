"""The agents' asyncio HTTP/1.1 server (api/server.py) and the gateway's pooled proxy client
(api/proxy.py): keep-alive, pipelining, chunked bodies both ways, limits, stale-connection retry."""
import asyncio
import socket

from starlette.applications import Starlette
from starlette.requests import Request
from starlette.responses import PlainTextResponse, Response, StreamingResponse
from starlette.routing import Route

from docagents_amd.api.proxy import PooledHTTPClient
from docagents_amd.api.server import serve


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _echo(req: Request):
    body = await req.body()
    return Response(body[::-1], status_code=201, headers={"x-path": req.url.path, "x-q": req.url.query},
                    media_type="application/octet-stream")


async def _stream(req):
    async def gen():
        for i in range(3):
            yield f"part{i};".encode()
    return StreamingResponse(gen(), media_type="text/plain")


async def _boom(req):
    raise RuntimeError("boom")


APP = Starlette(routes=[Route("/echo", _echo, methods=["POST"]), Route("/stream", _stream, methods=["GET", "POST"]),
                        Route("/boom", _boom), Route("/hi", lambda r: PlainTextResponse("hi"))])


async def _with_server(fn, max_body=1 << 20):
    port = _port()
    task = asyncio.create_task(serve(APP, "127.0.0.1", port, max_body=max_body))
    for _ in range(100):
        try:
            _, w = await asyncio.open_connection("127.0.0.1", port)
            w.close()
            break
        except OSError:
            await asyncio.sleep(0.02)
    try:
        return await fn(port)
    finally:
        task.cancel()


async def _raw(port, data: bytes, until_close=False, n_responses=1) -> bytes:
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(data)
    await w.drain()
    out = b""
    if until_close:
        out = await asyncio.wait_for(r.read(), 5)
    else:
        for _ in range(n_responses):
            head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
            n = int([ln.split(b":")[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
            out += head + await r.readexactly(n)
    w.close()
    return out


def test_keepalive_pipelined_and_query_string():
    async def go(port):
        req = b"POST /echo?a=1 HTTP/1.1\r\nHost: x\r\nContent-Length: 3\r\n\r\nabc"
        out = await _raw(port, req + req.replace(b"abc", b"xyz"), n_responses=2)
        assert out.count(b"HTTP/1.1 201 Created") == 2
        assert b"cba" in out and b"zyx" in out and b"x-q: a=1" in out
    asyncio.run(_with_server(go))


def test_chunked_request_stream_response_close_and_errors():
    async def go(port):
        out = await _raw(port, b"POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
                               b"3\r\nabc\r\n2\r\nde\r\n0\r\n\r\n")
        assert out.endswith(b"edcba")
        out = await _raw(port, b"GET /stream HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n", until_close=True)
        assert b"transfer-encoding: chunked" in out.lower() and b"part0;" in out and out.endswith(b"0\r\n\r\n")
        out = await _raw(port, b"GET /hi HTTP/1.0\r\n\r\n", until_close=True)
        assert out.startswith(b"HTTP/1.1 200") and out.endswith(b"hi")
        out = await _raw(port, b"POST /echo HTTP/1.1\r\nHost: x\r\nContent-Length: 99999999\r\n\r\n", until_close=True)
        assert out.startswith(b"HTTP/1.1 413")
        out = await _raw(port, b"GET /boom HTTP/1.1\r\nHost: x\r\n\r\n", until_close=True)
        assert out.startswith(b"HTTP/1.1 500")
    asyncio.run(_with_server(go))


def test_pooled_proxy_client_reuse_and_stale_retry():
    async def go(port):
        c = PooledHTTPClient(timeout=5)
        url = f"http://127.0.0.1:{port}/echo"
        for i in range(5):
            st, body = await c.post(url, f"hello{i}".encode(), {"Content-Type": "application/json"})
            assert st == 201 and body == f"hello{i}".encode()[::-1]
        key = ("127.0.0.1", port)
        assert len(c._idle[key]) == 1  # one connection reused for all five
        c._idle[key][0][1].close()  # simulate the server dropping the idle connection
        await asyncio.sleep(0.05)
        st, body = await c.post(url, b"again", {})
        assert st == 201 and body == b"niaga"
        st, body = await c.post(f"http://127.0.0.1:{port}/stream", b"", {})
        assert body == b"part0;part1;part2;"
        await c.aclose()
    asyncio.run(_with_server(go))
