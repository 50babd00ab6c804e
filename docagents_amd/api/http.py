"""HTTP plumbing with the reference's wire behaviour (internal/httputil/httputil.go).

* ``write_json``  — Go encoder output (sorted keys, 2-space indent, trailing newline), 200/202/...
* ``fail``        — ``http.Error``: ``text/plain; charset=utf-8``, ``X-Content-Type-Options: nosniff``,
                    body ``message\\n`` (httputil.go:102-108). Error bodies are NOT JSON.
* middleware chain (httputil.go:25-34), as pure ASGI: RequestID (``X-Request-Id``), RealIP,
  Timeout(60s -> 504), Recoverer (500 ``Internal Server Error``), RequestLogger (method, path,
  status, bytes, duration_ms, request_id). The request id is also exposed to handlers
  (``request.state.request_id``) and propagated into queue tasks / proxied requests (tracing).
* Prometheus ``/metrics`` (request latency histogram per route + status).
"""
from __future__ import annotations

import asyncio
import itertools
import os
import socket
import time
import traceback

from starlette.responses import Response

from . import gojson

try:
    from prometheus_client import Counter, Histogram
    REQ_LAT = Histogram("da_http_request_seconds", "HTTP request latency", ["service", "method", "route", "status"],
                        buckets=(0.0005, 0.001, 0.005, 0.01, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60))
    REQ_CNT = Counter("da_http_requests_total", "HTTP requests", ["service", "method", "route", "status"])
except Exception:  # pragma: no cover
    REQ_LAT = REQ_CNT = None


def write_json(status: int, body) -> Response:
    return Response(gojson.dumps(body), status_code=status, media_type="application/json")


def fail(log, message: str, err=None, status: int = 500) -> Response:
    if log is not None:
        log.error(message, "err", None if err is None else str(err))
    if status == 0:
        status = 500
    return Response(message + "\n", status_code=status,
                    headers={"content-type": "text/plain; charset=utf-8", "x-content-type-options": "nosniff"})


_host = socket.gethostname() or "localhost"
_prefix = f"{_host}/{os.urandom(5).hex()}"
_seq = itertools.count(1)


def new_request_id() -> str:
    return f"{_prefix}-{next(_seq):06d}"


class Middleware:
    """ASGI middleware implementing the reference's chi stack."""

    def __init__(self, app, log, service: str = "", timeout: float = 60.0):
        self.app, self.log, self.service, self.timeout = app, log, service, timeout

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        headers = {k.decode("latin-1").lower(): v.decode("latin-1") for k, v in scope.get("headers", [])}
        rid = headers.get("x-request-id") or new_request_id()
        state = scope.setdefault("state", {})
        state["request_id"] = rid
        real_ip = headers.get("true-client-ip") or headers.get("x-real-ip")
        if not real_ip and headers.get("x-forwarded-for"):
            real_ip = headers["x-forwarded-for"].split(",")[0].strip()
        if real_ip:
            scope["client"] = (real_ip, 0)
        start = time.perf_counter()
        info = {"status": 0, "bytes": 0, "started": False}

        async def _send(msg):
            if msg["type"] == "http.response.start":
                info["status"] = msg["status"]
                info["started"] = True
                hdrs = list(msg.get("headers", []))
                hdrs.append((b"x-request-id", rid.encode("latin-1")))
                msg = dict(msg, headers=hdrs)
            elif msg["type"] == "http.response.body":
                info["bytes"] += len(msg.get("body", b""))
            await send(msg)

        try:
            await asyncio.wait_for(self.app(scope, receive, _send), timeout=self.timeout)
        except asyncio.TimeoutError:
            if not info["started"]:
                await _send_plain(_send, 504, "Gateway Timeout")
        except Exception as e:  # noqa: BLE001 - Recoverer
            self.log.error("panic recovered", "panic", str(e), "path", scope.get("path"), "method", scope.get("method"),
                           "request_id", rid, "trace", traceback.format_exc(limit=5))
            if not info["started"]:
                await _send_plain(_send, 500, "Internal Server Error")
        dur = time.perf_counter() - start
        self.log.info("request", "method", scope.get("method"), "path", scope.get("path"), "status", info["status"],
                      "bytes", info["bytes"], "duration_ms", int(dur * 1000), "request_id", rid)
        if REQ_LAT is not None:
            route = scope.get("route_name") or _route_of(scope.get("path", ""))
            lbl = (self.service, scope.get("method", ""), route, str(info["status"]))
            REQ_LAT.labels(*lbl).observe(dur)
            REQ_CNT.labels(*lbl).inc()


def _route_of(path: str) -> str:
    parts = path.split("/")
    return "/".join("{id}" if len(p) == 36 and p.count("-") == 4 else p for p in parts)


async def _send_plain(send, status: int, text: str):
    body = (text + "\n").encode()
    await send({"type": "http.response.start", "status": status,
                "headers": [(b"content-type", b"text/plain; charset=utf-8"), (b"x-content-type-options", b"nosniff"),
                            (b"content-length", str(len(body)).encode())]})
    await send({"type": "http.response.body", "body": body})


def request_id(request) -> str:
    try:
        return request.scope["state"]["request_id"]
    except Exception:  # noqa: BLE001
        return ""


def metrics_response() -> Response:
    from prometheus_client import CONTENT_TYPE_LATEST, generate_latest
    return Response(generate_latest(), media_type=CONTENT_TYPE_LATEST)
