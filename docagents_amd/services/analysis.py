"""Analysis agent (cmd/analysis/main.go:57-122).

Order kept exactly: ListChunks -> concatenate -> LLM.Summarize -> SaveSummary -> GetDocument ->
enrich "Document: {filename}\\n\\n{chunk}" -> Embedder.EmbedBatch -> SaveEmbeddings -> status ready.
With the engine as both embedder and vector store, EmbedBatch + SaveEmbeddings are one engine step
(``embed_index``: vectors written into the owner shard's HBM, durably logged there).
Extras: the chunks' decoder token ids are cached for Answer prompts when the LLM runs on this
node, the 1:1 embedding mapping is enforced (the reference can index past the end, §5.3), and a
permanently failed analyze marks the document ``failed`` (the reference leaves it processing).
"""
from __future__ import annotations

import json
import uuid

from ..engine.prompts import concatenate_chunks, dedup_overlap, enrich_for_embedding
from ..queue.task import Task
from ..store.base import STATUS_FAILED, STATUS_READY, Embedding, Summary


async def handle_analyze(deps, payload: dict) -> None:
    doc_id = str(uuid.UUID(payload.get("document_id", "")))
    if payload.get("redrive"):
        # a startup-sweep re-drive of a document that finished meanwhile is a no-op (plain tasks keep
        # the reference's exact call order: ListChunks first)
        try:
            if (await deps.store.get_document(doc_id)).status == STATUS_READY:
                return
        except Exception:  # noqa: BLE001 - a missing document fails below, as before
            pass
    chunks = await deps.store.list_chunks(doc_id)
    # ord-ordered chunks with the sliding-window overlap removed: each word span summarized once
    text = concatenate_chunks(dedup_overlap([c.text for c in chunks], deps.config.chunk_overlap))
    summary, key_points = await deps.llm.summarize(text)
    await deps.store.save_summary(doc_id, Summary(doc_id, summary, key_points))
    try:
        doc = await deps.store.get_document(doc_id)
    except Exception as e:  # noqa: BLE001
        raise RuntimeError(f"failed to get document: {e}") from e
    texts = [enrich_for_embedding(doc.filename, c.text) for c in chunks]
    if getattr(deps.store, "direct_embed", False) is True:
        # engine embedder + engine vector shards: EmbedBatch and SaveEmbeddings in one engine step,
        # the vectors go from the encoder straight into the owner shard's HBM (no round trip)
        try:
            n = await deps.store.embed_and_save(doc_id, chunks, texts, deps.config.embedding_model)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"failed to generate embeddings: {e}") from e
        if n != len(chunks):
            raise RuntimeError(f"expected {len(chunks)} embeddings, got {n}")
    else:
        try:
            vectors = await deps.embedder.embed_batch(texts)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"failed to generate embeddings: {e}") from e
        if len(vectors) != len(chunks):
            raise RuntimeError(f"expected {len(chunks)} embeddings, got {len(vectors)}")
        embs = [Embedding(c.id, v, deps.config.embedding_model) for c, v in zip(chunks, vectors)]
        await deps.store.save_embeddings(embs)
    tok = deps.extras.get("dec_tokenizer")
    if tok is not None and chunks and hasattr(deps.store, "save_chunk_tokens"):
        enc = tok.encode_batch([c.text for c in chunks], add_special_tokens=False)
        await deps.store.save_chunk_tokens([(c.id, e.ids) for c, e in zip(chunks, enc)])
    await deps.store.update_document_status(doc_id, STATUS_READY)


def make_handler(deps):
    async def handler(task: Task):
        await handle_analyze(deps, json.loads(task.payload or b"{}"))
    return handler


def make_failure_hook(deps):
    async def on_fail(task: Task, err):
        try:
            doc_id = json.loads(task.payload or b"{}").get("document_id")
            if doc_id:
                await deps.store.update_document_status(str(uuid.UUID(doc_id)), STATUS_FAILED)
        except Exception:  # noqa: BLE001
            pass
    return on_fail
