"""Gateway agent: public HTTP API (cmd/gateway/main.go).

Routes: POST /api/documents/upload, GET /api/documents/{id}/summary, POST /api/query (proxied to
the query agent), GET /healthz, GET /metrics. Upload validation, text / PDF extraction, document
creation and parse-task enqueue follow main.go:53-158 exactly (same status codes and messages).

Design changes (documented in SURVEY.md §5.3 / Appendix B):
  * claim check: the extracted text is stored as a blob and the parse task carries a reference
    plus the text only when it is small — so >1 MB documents no longer break the queue;
  * the proxy target is configurable (QUERY_SERVICE_URL) and the request id is propagated;
  * the summary response adds ``documentId`` (promised by README.md:211, missing in the code).
"""
from __future__ import annotations

import asyncio
import json
import os
import uuid

from starlette.applications import Starlette
from starlette.requests import Request
from starlette.responses import PlainTextResponse, Response
from starlette.routing import Route

from ..api.http import Middleware, fail, metrics_response, request_id, write_json
from ..queue.task import TASK_PARSE, Task, enqueue_with_retry
from ..store.base import STATUS_FAILED
from ..text import multipart
from ..text.pdf import extract_text as pdf_text
from ..utils import timeline

ALLOWED_TYPES = {"text/plain", "application/pdf"}
INLINE_PAYLOAD_MAX = 256 * 1024


def validate_uploaded_file(content_length: int, part: multipart.Part, max_size: int):
    """main.go:111-146 -> (content_type, status, error message)."""
    if content_length > max_size:
        return "", 400, f"file too large (max {max_size} bytes)"
    if part.size > max_size:
        return "", 400, f"file too large (max {max_size} bytes)"
    ct = part.content_type
    if ct == "":
        ext = os.path.splitext(part.filename or "")[1].lower()
        if ext == ".txt":
            ct = "text/plain"
        elif ext == ".pdf":
            ct = "application/pdf"
        else:
            return "", 400, "unsupported file type (only PDF and TXT allowed)"
    if ct not in ALLOWED_TYPES:
        return "", 400, "unsupported file type (only PDF and TXT allowed)"
    return ct, 0, None


def extract_text(filename: str, content: bytes, log) -> str:
    """main.go:210-221: .pdf -> PDF text (raw bytes on failure); anything else -> raw bytes."""
    if filename.lower().endswith(".pdf"):
        try:
            return pdf_text(content)
        except Exception as e:  # noqa: BLE001
            log.warn("pdf extraction failed, using raw bytes", "err", e, "filename", filename)
            return content.decode("utf-8", errors="replace")
    return content.decode("utf-8", errors="replace")


async def _fail_doc(deps, message, err, doc_id, status, mark_failed):
    log = deps.log.with_("document_id", doc_id)
    if mark_failed and doc_id:
        try:
            await deps.store.update_document_status(doc_id, STATUS_FAILED)
        except Exception as e:  # noqa: BLE001
            log.error("failed to mark document failed", "err", e)
    return fail(log, message, err, status)


async def upload_handler(deps, request: Request) -> Response:
    cfg = deps.config
    ctype = request.headers.get("content-type", "")
    clen = int(request.headers.get("content-length") or -1)
    # bounded read: never buffer more than 2x the limit (+1 MiB of multipart framing)
    limit = 2 * cfg.max_upload_size + (1 << 20)
    body = bytearray()
    async for chunk in request.stream():
        body += chunk
        if len(body) > limit:
            return fail(deps.log, f"file too large (max {cfg.max_upload_size} bytes)", None, 400)
    try:
        part = multipart.form_file(bytes(body), ctype, "file")
    except multipart.MultipartError as e:
        return fail(deps.log, "file is required", e, 400)
    _, status, msg = validate_uploaded_file(clen if clen >= 0 else len(body), part, cfg.max_upload_size)
    if msg:
        return fail(deps.log, msg, None, status)
    filename = part.filename or ""
    text = await asyncio.to_thread(extract_text, filename, part.data, deps.log)
    try:
        doc = await deps.store.create_document(filename)
    except Exception as e:  # noqa: BLE001
        return fail(deps.log, "failed to persist document", e, 500)
    try:
        payload = {"document_id": doc.id, "filename": filename, "content": text}
        if len(text.encode("utf-8")) > INLINE_PAYLOAD_MAX and hasattr(deps.store, "put_blob"):
            ref = await deps.store.put_blob(doc.id, text.encode("utf-8"))
            payload = {"document_id": doc.id, "filename": filename, "content": "", "content_ref": ref}
        body = json.dumps(payload, ensure_ascii=False, separators=(",", ":")).encode()
    except Exception as e:  # noqa: BLE001
        return await _fail_doc(deps, "marshal payload failed", e, doc.id, 500, True)
    task = Task(type=TASK_PARSE, payload=body, trace_id=request_id(request))
    try:
        await enqueue_with_retry(deps.queue, task, 3, 0.2)
    except Exception as e:  # noqa: BLE001
        return await _fail_doc(deps, "failed to enqueue document; please retry", e, doc.id, 500, True)
    return write_json(202, {"document_id": doc.id, "status": doc.status})


async def summary_handler(deps, id_str: str) -> Response:
    try:
        doc_id = str(uuid.UUID(id_str))
    except (ValueError, AttributeError) as e:
        return fail(deps.log, "invalid document id", e, 400)
    try:
        s = await deps.store.get_summary(doc_id)
    except Exception as e:  # noqa: BLE001 - ANY store error -> 404 (main.go:169-171)
        return fail(deps.log.with_("document_id", doc_id), "summary not ready", e, 404)
    return write_json(200, {"summary": s.summary, "key_points": list(s.key_points) if s.key_points is not None else None,
                            "documentId": doc_id})


async def query_proxy(deps, request: Request) -> Response:
    """main.go:180-207: forward the body verbatim; status + body back, Content-Type forced."""
    from ..api.proxy import PooledHTTPClient
    body = await request.body()
    q = None
    if timeline.enabled():
        try:
            q = json.loads(body).get("question")
        except (ValueError, AttributeError):
            pass
        timeline.mark("g_rx", q=q)
    client = deps.extras.get("http")
    if client is None:
        client = PooledHTTPClient(timeout=60.0)
        deps.extras["http"] = client
    try:
        status, content = await client.post(deps.config.query_service_url, body,
                                            {"Content-Type": "application/json", "X-Request-Id": request_id(request)})
    except Exception as e:  # noqa: BLE001
        return fail(deps.log, "query service unavailable", e, 503)
    if q is not None:
        timeline.mark("g_tx", q=q)
    return Response(content, status_code=status, media_type="application/json")


def build_app(deps) -> Middleware:
    async def upload(req):
        return await upload_handler(deps, req)

    async def summary(req):
        return await summary_handler(deps, req.path_params["id"])

    async def query(req):
        return await query_proxy(deps, req)

    async def health(req):
        return PlainTextResponse("ok")

    async def metrics(req):
        return metrics_response()

    app = Starlette(routes=[
        Route("/api/documents/upload", upload, methods=["POST"]),
        Route("/api/documents/{id}/summary", summary, methods=["GET"]),
        Route("/api/query", query, methods=["POST"]),
        Route("/healthz", health, methods=["GET"]),
        Route("/metrics", metrics, methods=["GET"]),
    ])
    return Middleware(app, deps.log, "gateway")
