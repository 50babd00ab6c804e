"""Parser agent (cmd/parser/main.go): consume ``parse`` tasks, chunk 400/80, save chunks, enqueue
``analyze``. ``save_chunks`` replaces the document's chunks in one transaction, so a retried parse
is idempotent."""
from __future__ import annotations

import json
import uuid

from ..queue.task import TASK_ANALYZE, Task, enqueue_with_retry
from ..store.base import Chunk
from ..text.chunker import Options, chunk_text


async def handle_parse(deps, payload: dict, trace_id: str = "") -> None:
    doc_id = str(uuid.UUID(payload.get("document_id", "")))
    text = payload.get("content") or ""
    if not text and payload.get("content_ref") and hasattr(deps.store, "get_blob"):
        text = (await deps.store.get_blob(payload["content_ref"])).decode("utf-8", errors="replace")
    cfg = deps.config
    chunks = chunk_text(text, Options(cfg.chunk_max_tokens, cfg.chunk_overlap))
    saved = await deps.store.save_chunks(doc_id, [Chunk(index=c.index, text=c.text, token_count=c.token_count)
                                                  for c in chunks])
    body = json.dumps({"document_id": doc_id, "chunk_ids": [c.id for c in saved] or None},
                      separators=(",", ":")).encode()
    await enqueue_with_retry(deps.queue, Task(type=TASK_ANALYZE, payload=body, trace_id=trace_id), 3, 0.2)


def make_handler(deps):
    async def handler(task: Task):
        payload = json.loads(task.payload or b"{}")
        await handle_parse(deps, payload, task.trace_id)
    return handler


def make_failure_hook(deps):
    """A parse task that exhausted its retries marks the document 'failed' (the reference leaves
    it 'processing' forever)."""
    async def on_fail(task: Task, err):
        try:
            doc_id = json.loads(task.payload or b"{}").get("document_id")
            if doc_id:
                await deps.store.update_document_status(str(uuid.UUID(doc_id)), "failed")
        except Exception:  # noqa: BLE001
            pass
    return on_fail
