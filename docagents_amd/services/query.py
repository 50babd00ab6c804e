"""Query agent (cmd/query/main.go:44-195): validate -> query cache -> embedding cache -> embed ->
TopK -> context -> LLM answer -> cache set -> respond.

Response: ``{"answer", "cached", "confidence" (float32), "sources": [{"chunk_id","score","preview"}]}``
with the reference's status codes and messages. confidence = avg similarity x mean token
probability of the answer (llm/openai.go:101-102); preview = first 150 bytes cut at a word.
"""
from __future__ import annotations

import asyncio
import time
import uuid

import numpy as np
from starlette.applications import Starlette
from starlette.requests import Request
from starlette.responses import PlainTextResponse, Response
from starlette.routing import Route

from ..api.gojson import F32
from ..api.http import Middleware, fail, metrics_response, write_json
from ..api.validation import PayloadError, decode_query_request, validate_query_request
from ..cache.cache import QueryResult, Source
from ..cache.keys import generate_cache_key
from ..providers import EmbedError
from ..text.preprocess import preprocess_text, truncate_preview
from ..utils import timeline

try:
    from prometheus_client import Counter, Histogram
    CACHE_OUT = Counter("da_query_cache_total", "query cache outcomes", ["outcome"])
    STAGE = Histogram("da_query_stage_seconds", "query stage latency", ["stage"],
                      buckets=(0.0005, 0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5))
except Exception:  # pragma: no cover
    CACHE_OUT = STAGE = None


def _obs(stage, t0):
    if STAGE is not None:
        STAGE.labels(stage).observe(time.perf_counter() - t0)


def parse_document_ids(ids: list[str]) -> list[str]:
    out = []
    for s in ids:
        try:
            out.append(str(uuid.UUID(s)))
        except (ValueError, AttributeError):
            continue
    return out


def build_context(results) -> str:
    return "".join(r.chunk.text + "\n" for r in results)


def calculate_avg_similarity(results) -> float:
    if not results:
        return 0.0
    s = np.float32(0.0)
    for r in results:
        s = np.float32(s + np.float32(r.score))
    return float(np.float32(s / np.float32(len(results))))


def build_sources(results) -> list[Source]:
    return [Source(r.chunk.id, float(np.float32(r.score)), truncate_preview(r.chunk.text, 150)) for r in results]


_BG: set = set()


def _background(coro):
    """Run ``coro`` without awaiting it (a reference is kept until it finishes)."""
    t = asyncio.ensure_future(coro)
    _BG.add(t)
    t.add_done_callback(_BG.discard)


async def _set_embedding(deps, question, vec, ttl, log):
    try:
        await deps.cache.set_embedding(question, vec, ttl)
    except Exception as e:  # noqa: BLE001
        log.warn("failed to cache embedding", "err", e)


def _resp(answer, sources, confidence, cached):
    return {"answer": answer, "sources": [s.to_json() for s in sources], "confidence": F32(confidence),
            "cached": cached}


async def query_handler(deps, body: bytes) -> Response:
    log = deps.log
    try:
        req = decode_query_request(body)
    except PayloadError as e:
        return fail(log, "invalid payload", e, 400)
    msgs = validate_query_request(req)
    if msgs:
        return fail(log, "; ".join(msgs), None, 400)
    if req.top_k == 0:
        req.top_k = 5
    t0 = time.perf_counter()
    if timeline.enabled():
        timeline.mark("q_start", q=req.question)
    key = generate_cache_key(req.question, req.document_ids, req.top_k)
    try:
        cached = await deps.cache.get_query_result(key)
    except Exception:  # noqa: BLE001 - GET error falls through as a miss
        cached = None
    if cached is not None:
        log.info("cache hit", "question", req.question)
        if CACHE_OUT is not None:
            CACHE_OUT.labels("hit").inc()
        _obs("cache_hit", t0)
        return write_json(200, _resp(cached.answer, cached.sources, cached.confidence, True))
    if CACHE_OUT is not None:
        CACHE_OUT.labels("miss").inc()
    ids = parse_document_ids(req.document_ids)
    vec = None
    try:
        vec = await deps.cache.get_embedding(req.question)
    except Exception as e:  # noqa: BLE001
        log.warn("failed to get cached embedding", "err", e)
    ttl = deps.config.cache_ttl
    results = None
    if vec is None and getattr(deps.store, "fused_query", False) is True:
        # embed + search in one engine call (the reference's two calls, main.go:88 + :101)
        text = preprocess_text(req.question)
        if not text:
            return fail(log, "failed to embed question", EmbedError("text is empty after preprocessing"), 500)
        t1 = time.perf_counter()
        try:
            vec, results = await deps.store.embed_top_k(ids, text, req.top_k)
        except Exception as e:  # noqa: BLE001
            # the engine tags which half failed (engine/server.py embed_search)
            msg = "search failed" if "embed_search/search:" in str(e) else "failed to embed question"
            return fail(log, msg, e, 500)
        _obs("embed_search", t1)
        if timeline.enabled():
            timeline.mark("q_searched", q=req.question)
        # not awaited: the answer does not need it, and the cache client is pipelined over one
        # connection, so this SET still reaches the cache before the query-result SET below (the
        # reference's visibility: both are in the cache when the response is written)
        _background(_set_embedding(deps, req.question, vec, ttl, log))
        if timeline.enabled():
            timeline.mark("q_embed_cached", q=req.question)
    if vec is None:
        t1 = time.perf_counter()
        try:
            vec = await deps.embedder.embed(req.question)
        except Exception as e:  # noqa: BLE001
            return fail(log, "failed to embed question", e, 500)
        _obs("embed", t1)
        try:
            await deps.cache.set_embedding(req.question, vec, ttl)
        except Exception as e:  # noqa: BLE001
            log.warn("failed to cache embedding", "err", e)
    if results is None:
        t2 = time.perf_counter()
        try:
            results = await deps.store.top_k(ids, vec, req.top_k)
        except Exception as e:  # noqa: BLE001
            return fail(log, "search failed", e, 500)
        _obs("search", t2)
    context = build_context(results)
    quality = calculate_avg_similarity(results)
    t3 = time.perf_counter()
    if timeline.enabled():
        timeline.mark("q_answer_sent", q=req.question)
    try:
        if getattr(deps.llm, "supports_chunks", False) and hasattr(deps.store, "chunks_by_keys") and results:
            if all(getattr(r, "tokens_loaded", False) for r in results):  # read with the hits
                blobs = [r.tokens for r in results]
            else:
                toks = await deps.store.chunks_by_keys([r.chunk.key for r in results])
                blobs = [toks.get(r.chunk.key, (None, None))[1] for r in results]
            # token ids stay an int32 array (the engine RPC ships it as one buffer): no per-token
            # Python ints on the query path
            chunks = [(r.chunk.text, np.frombuffer(b, dtype=np.int32) if b else None)
                      for r, b in zip(results, blobs)]
            answer, confidence = await deps.llm.answer_chunks(req.question, chunks, quality)
        else:
            answer, confidence = await deps.llm.answer(req.question, context, quality)
    except Exception as e:  # noqa: BLE001
        return fail(log, "llm failed", e, 500)
    _obs("answer", t3)
    if timeline.enabled():
        timeline.mark("q_answer_rx", q=req.question)
    sources = build_sources(results)
    try:
        await deps.cache.set_query_result(key, QueryResult(answer, confidence, sources), ttl)
    except Exception as e:  # noqa: BLE001
        log.warn("failed to cache result", "err", e)
    _obs("cache_miss_total", t0)
    if timeline.enabled():
        timeline.mark("q_end", q=req.question)
    return write_json(200, _resp(answer, sources, confidence, False))


def build_app(deps) -> Middleware:
    async def query(req: Request):
        return await query_handler(deps, await req.body())

    async def health(req):
        return PlainTextResponse("ok")

    async def metrics(req):
        return metrics_response()

    app = Starlette(routes=[Route("/api/query", query, methods=["POST"]), Route("/healthz", health, methods=["GET"]),
                            Route("/metrics", metrics, methods=["GET"])])
    return Middleware(app, deps.log, "query")
