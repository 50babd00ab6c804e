"""Agent parity tests, ported from cmd/gateway/main_test.go, cmd/query/main_test.go,
cmd/analysis/main_test.go and cmd/parser/main_test.go (testify mocks -> call-recording fakes)."""
import asyncio
import json
import uuid

import numpy as np
import pytest
from starlette.testclient import TestClient

from docagents_amd.app import Deps
from docagents_amd.cache.cache import MemoryCache
from docagents_amd.config import Config
from docagents_amd.services import analysis, gateway, parser, query
from docagents_amd.store.base import Chunk, Document, SearchResult, Summary, SummaryNotFound
from docagents_amd.text import multipart
from docagents_amd.text.pdf import make_pdf
from docagents_amd.utils.log import discard


class Spy:
    """Records calls; behaviour per method from a dict of callables / values / exceptions."""

    def __init__(self, **behaviour):
        self.calls = []
        self.b = behaviour

    def __getattr__(self, name):
        if name.startswith("__") or name.startswith("supports_"):
            raise AttributeError(name)

        async def fn(*a, **k):
            self.calls.append((name, a))
            v = self.b.get(name)
            if isinstance(v, Exception):
                raise v
            if callable(v):
                return v(*a)
            return v
        return fn

    def names(self):
        return [c[0] for c in self.calls]


def deps_for(**kw):
    d = Deps(Config(max_upload_size=1024 * 1024, embedding_model="test-model", cache_ttl=86400), discard())
    for k, v in kw.items():
        setattr(d, k, v)
    return d


DOC = str(uuid.uuid4())


# ======================================================================= gateway upload
def _upload(client, filename, data, ctype):
    body, ct = multipart.build({}, {"file": (filename, data, ctype)})
    return client.post("/api/documents/upload", content=body, headers={"content-type": ct})


def test_upload_success():
    store = Spy(create_document=Document(DOC, "test.txt"))
    q = Spy(enqueue=None)
    c = TestClient(gateway.build_app(deps_for(store=store, queue=q)))
    r = _upload(c, "test.txt", b"This is test content", "text/plain")
    assert r.status_code == 202
    assert r.json() == {"document_id": DOC, "status": "processing"}
    task = q.calls[0][1][0]
    assert task.type == "parse"
    p = json.loads(task.payload)
    assert p == {"document_id": DOC, "filename": "test.txt", "content": "This is test content"}


def test_upload_too_large():
    c = TestClient(gateway.build_app(deps_for(store=Spy(), queue=Spy())))
    r = _upload(c, "big.txt", b"x" * (1024 * 1024 + 1), "text/plain")
    assert r.status_code == 400 and r.text == "file too large (max 1048576 bytes)\n"


def test_upload_detects_type_from_extension():
    store = Spy(create_document=Document(DOC, "notes.txt"))
    c = TestClient(gateway.build_app(deps_for(store=store, queue=Spy(enqueue=None))))
    assert _upload(c, "notes.txt", b"hello", None).status_code == 202


@pytest.mark.parametrize("fn,ct", [("file.docx", None), ("file.doc", "application/msword")])
def test_upload_unsupported(fn, ct):
    c = TestClient(gateway.build_app(deps_for(store=Spy(), queue=Spy())))
    r = _upload(c, fn, b"x", ct)
    assert r.status_code == 400 and r.text == "unsupported file type (only PDF and TXT allowed)\n"
    assert r.headers["content-type"] == "text/plain; charset=utf-8"


def test_upload_store_error():
    c = TestClient(gateway.build_app(deps_for(store=Spy(create_document=RuntimeError("db")), queue=Spy())))
    r = _upload(c, "a.txt", b"x", "text/plain")
    assert r.status_code == 500 and r.text == "failed to persist document\n"


def test_upload_enqueue_fails_three_times_marks_failed(monkeypatch):
    async def no_sleep(_):
        return None
    monkeypatch.setattr(asyncio, "sleep", no_sleep)
    store = Spy(create_document=Document(DOC, "a.txt"), update_document_status=None)
    q = Spy(enqueue=RuntimeError("queue down"))
    c = TestClient(gateway.build_app(deps_for(store=store, queue=q)))
    r = _upload(c, "a.txt", b"x", "text/plain")
    assert r.status_code == 500 and r.text == "failed to enqueue document; please retry\n"
    assert q.names().count("enqueue") == 3
    assert ("update_document_status", (DOC, "failed")) in store.calls


def test_upload_missing_file():
    c = TestClient(gateway.build_app(deps_for(store=Spy(), queue=Spy())))
    r = c.post("/api/documents/upload", content=b"{}", headers={"content-type": "application/json"})
    assert r.status_code == 400 and r.text == "file is required\n"


def test_upload_pdf_extracts_text():
    store = Spy(create_document=Document(DOC, "doc.pdf"))
    q = Spy(enqueue=None)
    c = TestClient(gateway.build_app(deps_for(store=store, queue=q)))
    r = _upload(c, "doc.pdf", make_pdf(["Hello PDF world"]), "application/pdf")
    assert r.status_code == 202
    assert json.loads(q.calls[0][1][0].payload)["content"] == "Hello PDF world\n"


def test_upload_bad_pdf_falls_back_to_raw():
    store = Spy(create_document=Document(DOC, "doc.pdf"))
    q = Spy(enqueue=None)
    c = TestClient(gateway.build_app(deps_for(store=store, queue=q)))
    assert _upload(c, "doc.pdf", b"not really a pdf", "application/pdf").status_code == 202
    assert json.loads(q.calls[0][1][0].payload)["content"] == "not really a pdf"


# ======================================================================= gateway summary
def test_summary_success():
    store = Spy(get_summary=Summary(DOC, "Test summary", ["Point 1", "Point 2"]))
    c = TestClient(gateway.build_app(deps_for(store=store)))
    r = c.get(f"/api/documents/{DOC}/summary")
    assert r.status_code == 200
    assert r.json() == {"summary": "Test summary", "key_points": ["Point 1", "Point 2"], "documentId": DOC}
    assert r.text.startswith('{\n  "documentId"')


@pytest.mark.parametrize("err,code,msg", [(SummaryNotFound(), 404, "summary not ready\n"),
                                          (RuntimeError("database connection failed"), 404, "summary not ready\n")])
def test_summary_errors(err, code, msg):
    c = TestClient(gateway.build_app(deps_for(store=Spy(get_summary=err))))
    r = c.get(f"/api/documents/{DOC}/summary")
    assert r.status_code == code and r.text == msg


def test_summary_bad_uuid():
    c = TestClient(gateway.build_app(deps_for(store=Spy())))
    r = c.get("/api/documents/not-a-uuid/summary")
    assert r.status_code == 400 and r.text == "invalid document id\n"


def test_healthz_and_request_id():
    c = TestClient(gateway.build_app(deps_for()))
    r = c.get("/healthz", headers={"X-Request-Id": "abc"})
    assert r.status_code == 200 and r.text == "ok" and r.headers["x-request-id"] == "abc"


# ======================================================================= query agent
def q_deps(results=None, answer=("Go is a programming language developed by Google", 0.95), cache=None,
           topk_err=None, llm_err=None):
    emb = Spy(embed=np.array([0.1, 0.2], dtype=np.float32))
    store = Spy(top_k=topk_err if topk_err else (results if results is not None else []))
    llm = Spy(answer=llm_err if llm_err else answer)
    return deps_for(embedder=emb, store=store, llm=llm, cache=cache or MemoryCache()), emb, store, llm


def _q(c, body):
    return c.post("/api/query", content=json.dumps(body) if not isinstance(body, str) else body)


def test_query_full_miss_path_and_cache_hit():
    cid = str(uuid.uuid4())
    res = [SearchResult(Chunk(cid, DOC, 0, "Go is a programming language", 5), 0.95, Summary())]
    d, emb, store, llm = q_deps(res)
    c = TestClient(query.build_app(d))
    r = _q(c, {"question": "What is Go?", "document_ids": [DOC], "top_k": 3})
    assert r.status_code == 200
    j = r.json()
    assert j["cached"] is False and j["answer"].startswith("Go is")
    assert j["sources"] == [{"chunk_id": cid, "score": 0.95, "preview": "Go is a programming language"}]
    assert emb.calls == [("embed", ("What is Go?",))]
    assert store.calls[0][0] == "top_k" and store.calls[0][1][0] == [DOC] and store.calls[0][1][2] == 3
    q_, ctx, quality = llm.calls[0][1]
    assert q_ == "What is Go?" and ctx == "Go is a programming language\n" and abs(quality - 0.95) < 1e-6
    # second identical request: full cache hit, no embed / search / llm
    r2 = _q(c, {"question": "What is Go?", "document_ids": [DOC], "top_k": 3})
    assert r2.json()["cached"] is True and r2.json()["answer"] == j["answer"]
    assert len(emb.calls) == 1 and len(llm.calls) == 1
    # key order of the Go map response
    assert r.text.index('"answer"') < r.text.index('"cached"') < r.text.index('"confidence"') < r.text.index('"sources"')


def test_query_embedding_cache_partial_hit():
    cache = MemoryCache()
    d, emb, store, llm = q_deps([], cache=cache)
    c = TestClient(query.build_app(d))
    _q(c, {"question": "What is Go?", "document_ids": [DOC]})
    _q(c, {"question": "What is Go?", "document_ids": [DOC], "top_k": 7})  # different key, same question
    assert len(emb.calls) == 1 and len(llm.calls) == 2


def test_query_top_k_default_5_and_empty_results():
    d, emb, store, llm = q_deps([], answer=("I don't have enough context", 0.3))
    c = TestClient(query.build_app(d))
    r = _q(c, {"question": "What is Go?", "document_ids": [DOC]})
    assert r.status_code == 200 and r.json()["sources"] == []
    assert store.calls[0][1][2] == 5
    assert llm.calls[0][1] == ("What is Go?", "", 0.0)


@pytest.mark.parametrize("body,code", [("{invalid json}", 400), ({"question": "", "document_ids": [DOC]}, 400),
                                       ({"question": "Hi", "document_ids": [DOC]}, 400),
                                       ({"question": "Valid question here", "document_ids": ["not-a-uuid"]}, 400),
                                       ({"question": "Valid question", "document_ids": []}, 400),
                                       ({"question": "Valid question", "document_ids": [DOC], "top_k": 25}, 400)])
def test_query_validation(body, code):
    d, emb, store, llm = q_deps()
    r = _q(TestClient(query.build_app(d)), body)
    assert r.status_code == code and not emb.calls and not llm.calls
    if body == "{invalid json}":
        assert r.text == "invalid payload\n"


def test_query_topk_error_and_llm_error():
    d, *_ = q_deps(topk_err=RuntimeError("database error"))
    r = _q(TestClient(query.build_app(d)), {"question": "What is Go?", "document_ids": [DOC]})
    assert r.status_code == 500 and r.text == "search failed\n"
    d, *_ = q_deps(llm_err=RuntimeError("LLM error"))
    r = _q(TestClient(query.build_app(d)), {"question": "What is Go?", "document_ids": [DOC]})
    assert r.status_code == 500 and r.text == "llm failed\n"


def test_query_embed_error():
    d, emb, *_ = q_deps()
    emb.b["embed"] = RuntimeError("boom")
    r = _q(TestClient(query.build_app(d)), {"question": "What is Go?", "document_ids": [DOC]})
    assert r.status_code == 500 and r.text == "failed to embed question\n"


def test_avg_similarity_and_sources():
    rs = [SearchResult(Chunk("a", text="x " * 200), 0.9, Summary()), SearchResult(Chunk("b", text="y"), 0.7, Summary())]
    assert abs(query.calculate_avg_similarity(rs) - 0.8) < 1e-6
    assert query.calculate_avg_similarity([]) == 0.0
    src = query.build_sources(rs)
    assert src[0].preview.endswith("...") and src[1].preview == "y"


# ======================================================================= analysis agent
def a_deps(chunks, summarize=("Test summary", ["Key point 1"]), **over):
    store = Spy(list_chunks=chunks, save_summary=None, get_document=Document(DOC, "test.pdf"),
                save_embeddings=None, update_document_status=None)
    llm = Spy(summarize=summarize)
    emb = Spy(embed_batch=lambda texts: [np.ones(3, dtype=np.float32) for _ in texts])
    for k, v in over.items():
        {"store": store, "llm": llm, "emb": emb}[k.split("_", 1)[0]].b[k.split("_", 1)[1]] = v
    return deps_for(store=store, llm=llm, embedder=emb), store, llm, emb


def test_analysis_call_order_single_chunk():
    c1 = str(uuid.uuid4())
    d, store, llm, emb = a_deps([Chunk(c1, DOC, 0, "Test chunk", 2)])
    asyncio.run(analysis.handle_analyze(d, {"document_id": DOC, "chunk_ids": [c1]}))
    assert llm.calls == [("summarize", ("Test chunk\n",))]
    assert emb.calls == [("embed_batch", (["Document: test.pdf\n\nTest chunk"],))]
    assert store.names() == ["list_chunks", "save_summary", "get_document", "save_embeddings",
                             "update_document_status"]
    embs = store.calls[3][1][0]
    assert len(embs) == 1 and embs[0].chunk_id == c1 and embs[0].model == "test-model"
    assert store.calls[4][1] == (DOC, "ready")


def test_analysis_multi_chunk_concat():
    d, store, llm, emb = a_deps([Chunk("a", DOC, 0, "First chunk", 2), Chunk("b", DOC, 1, "Second chunk", 2)])
    asyncio.run(analysis.handle_analyze(d, {"document_id": DOC}))
    assert llm.calls[0][1] == ("First chunk\nSecond chunk\n",)


def test_analysis_bad_uuid():
    d, store, *_ = a_deps([])
    with pytest.raises(ValueError):
        asyncio.run(analysis.handle_analyze(d, {"document_id": "invalid-uuid"}))
    assert not store.calls


@pytest.mark.parametrize("over,stop_before", [
    ({"store_list_chunks": RuntimeError("db")}, "save_summary"),
    ({"llm_summarize": RuntimeError("llm")}, "get_document"),
    ({"store_save_summary": RuntimeError("db")}, "get_document"),
    ({"store_get_document": RuntimeError("nf")}, "save_embeddings"),
    ({"emb_embed_batch": RuntimeError("emb")}, "save_embeddings"),
    ({"store_save_embeddings": RuntimeError("db")}, "update_document_status"),
])
def test_analysis_failures_propagate(over, stop_before):
    d, store, llm, emb = a_deps([Chunk("a", DOC, 0, "x", 1)], **over)
    with pytest.raises(Exception):
        asyncio.run(analysis.handle_analyze(d, {"document_id": DOC}))
    assert stop_before not in store.names()


def test_analysis_empty_chunks_still_ready():
    d, store, llm, emb = a_deps([])
    asyncio.run(analysis.handle_analyze(d, {"document_id": DOC}))
    assert llm.calls == [("summarize", ("",))]
    assert emb.calls == [("embed_batch", ([],))]
    assert store.calls[3] == ("save_embeddings", ([],)) and store.calls[4][1] == (DOC, "ready")


# ======================================================================= parser agent
def p_deps(**b):
    store = Spy(save_chunks=lambda doc, chunks: [Chunk(str(uuid.uuid4()), doc, c.index, c.text, c.token_count)
                                                 for c in chunks])
    store.b.update(b)
    q = Spy(enqueue=None)
    return deps_for(store=store, queue=q), store, q


def test_parse_small_text():
    d, store, q = p_deps()
    asyncio.run(parser.handle_parse(d, {"document_id": DOC, "filename": "t.txt", "content": "This is a test document."}))
    chunks = store.calls[0][1][1]
    assert len(chunks) >= 1 and chunks[0].text == "This is a test document."
    t = q.calls[0][1][0]
    assert t.type == "analyze" and json.loads(t.payload)["document_id"] == DOC


def test_parse_large_text_multiple_chunks():
    d, store, q = p_deps()
    asyncio.run(parser.handle_parse(d, {"document_id": DOC, "content": " ".join(["word"] * 1000)}))
    assert [c.token_count for c in store.calls[0][1][1]] == [400, 400, 360]


def test_parse_bad_uuid_and_errors():
    d, store, q = p_deps()
    with pytest.raises(ValueError):
        asyncio.run(parser.handle_parse(d, {"document_id": "invalid-uuid", "content": "x"}))
    d, store, q = p_deps(save_chunks=RuntimeError("db"))
    with pytest.raises(RuntimeError):
        asyncio.run(parser.handle_parse(d, {"document_id": DOC, "content": "x y"}))
    assert not q.calls


def test_parse_enqueue_error(monkeypatch):
    async def no_sleep(_):
        return None
    monkeypatch.setattr(asyncio, "sleep", no_sleep)
    d, store, q = p_deps()
    q.b["enqueue"] = RuntimeError("queue")
    with pytest.raises(RuntimeError):
        asyncio.run(parser.handle_parse(d, {"document_id": DOC, "content": "x y"}))
    assert q.names().count("enqueue") == 3


def test_parse_empty_content_still_enqueues():
    d, store, q = p_deps()
    asyncio.run(parser.handle_parse(d, {"document_id": DOC, "content": ""}))
    assert len(q.calls) == 1


def test_query_fused_embed_search_one_engine_call():
    """With the engine behind both the embedder and the vectors, a cache miss embeds and searches
    in ONE call (embed_top_k); the vector still lands in the embedding cache, and the next query
    with the same question (another document set) searches with the cached vector."""
    cid = str(uuid.uuid4())
    res = [SearchResult(Chunk(cid, DOC, 0, "Go is a programming language", 5), 0.9, Summary())]

    class Store(Spy):
        fused_query = True
    store = Store(embed_top_k=(np.array([0.6, 0.8], dtype=np.float32), res), top_k=res)
    emb = Spy(embed=np.array([0.1, 0.2], dtype=np.float32))
    llm = Spy(answer=("an answer", 0.9))
    cache = MemoryCache()
    c = TestClient(query.build_app(deps_for(embedder=emb, store=store, llm=llm, cache=cache)))
    r = _q(c, {"question": "  What\tis Go? ", "document_ids": [DOC], "top_k": 2})
    assert r.status_code == 200 and r.json()["sources"][0]["chunk_id"] == cid
    assert store.names() == ["embed_top_k"] and emb.calls == []
    assert store.calls[0][1] == ([DOC], "What is Go?", 2)  # preprocessed text, reference order of args
    other = str(uuid.uuid4())
    r2 = _q(c, {"question": "  What\tis Go? ", "document_ids": [other], "top_k": 2})
    assert r2.status_code == 200 and store.names() == ["embed_top_k", "top_k"]
    np.testing.assert_allclose(store.calls[1][1][1], [0.6, 0.8])
    # the engine's tag decides the reference's error message
    bad = Store(embed_top_k=RuntimeError("RPCError: RuntimeError: embed_search/search: shard down"))
    c2 = TestClient(query.build_app(deps_for(embedder=emb, store=bad, llm=llm, cache=MemoryCache())))
    r3 = _q(c2, {"question": "What is Go?", "document_ids": [DOC]})
    assert r3.status_code == 500 and r3.text == "search failed\n"
    bad2 = Store(embed_top_k=RuntimeError("RPCError: RuntimeError: embed_search/embed: boom"))
    c3 = TestClient(query.build_app(deps_for(embedder=emb, store=bad2, llm=llm, cache=MemoryCache())))
    assert _q(c3, {"question": "What is Go?", "document_ids": [DOC]}).text == "failed to embed question\n"
