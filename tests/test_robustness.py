"""Robustness: many concurrent uploads through competing parser/analysis workers (every document
processed exactly once, chunks never duplicated by a retried parse), injected faults
(DA_FAULT sites) recovered by the retry machinery, and permanent failure -> status 'failed'
(the reference leaves such documents 'processing' forever)."""
import asyncio
import datetime as dt
import json

from docagents_amd.app import Deps
from docagents_amd.config import Config
from docagents_amd.providers import StubEmbedder, StubLLM
from docagents_amd.queue import inproc as inproc_mod
from docagents_amd.queue.inproc import InProcBus, InProcQueue
from docagents_amd.queue.task import TASK_PARSE, Task
from docagents_amd.services import analysis, parser
from docagents_amd.store.sqlite_store import CompositeStore, SqliteMeta
from docagents_amd.store.sqlite_vectors import SqliteVectors
from docagents_amd.utils import faults
from docagents_amd.utils.log import discard


def _fast_retry(t, now=None):
    t.attempts += 1
    if t.max_attempts == 0:
        t.max_attempts = 5
    if t.attempts < t.max_attempts:
        t.not_before = dt.datetime.now(dt.timezone.utc) + dt.timedelta(milliseconds=2)
        return t
    return None


def _stack(tmp_path):
    meta = SqliteMeta(str(tmp_path / "m.sqlite3"))
    store = CompositeStore(meta, SqliteVectors(meta), min_similarity=-1.0)
    bus = InProcBus()
    d = Deps(Config(), discard(), store=store, queue=InProcQueue(bus, discard()), llm=StubLLM(),
             embedder=StubEmbedder(32))
    return d, bus


async def _run_workers(d, bus, n_workers, stop):
    ws = []
    for _ in range(n_workers):
        qp = InProcQueue(bus, discard())
        qa = InProcQueue(bus, discard())
        ws.append(asyncio.ensure_future(qp.worker("parse", parser.make_handler(d), stop,
                                                  on_permanent_failure=parser.make_failure_hook(d))))
        ws.append(asyncio.ensure_future(qa.worker("analyze", analysis.make_handler(d), stop,
                                                  on_permanent_failure=analysis.make_failure_hook(d))))
    return ws


def test_concurrent_uploads_exactly_once_with_faults(tmp_path, monkeypatch):
    monkeypatch.setattr(inproc_mod, "next_retry", _fast_retry)
    faults.configure({"handler.parse": 0.3, "handler.analyze": 0.3, "store.save_chunks": 0.2})
    try:
        async def go():
            d, bus = _stack(tmp_path)
            stop = asyncio.Event()
            ws = await _run_workers(d, bus, 3, stop)
            docs = []
            for i in range(40):
                doc = await d.store.create_document(f"f{i}.txt")
                docs.append(doc.id)
                body = json.dumps({"document_id": doc.id, "filename": f"f{i}.txt",
                                   "content": " ".join(f"w{i}_{j}" for j in range(900))}).encode()
                await d.queue.enqueue(Task(type=TASK_PARSE, payload=body))
            for _ in range(400):
                st = [(await d.store.get_document(x)).status for x in docs]
                if all(s != "processing" for s in st):
                    break
                await asyncio.sleep(0.05)
            stop.set()
            await asyncio.gather(*ws)
            return d, docs, st
        d, docs, statuses = asyncio.run(go())
    finally:
        faults.configure(None)

    async def check():
        n_ready = 0
        for x, s in zip(docs, statuses):
            chunks = await d.store.list_chunks(x)
            if s == "ready":
                n_ready += 1
                assert [c.index for c in chunks] == [0, 1, 2]  # 900 words -> 3 chunks, never duplicated
            else:
                assert s == "failed"
        return n_ready
    n_ready = asyncio.run(check())
    assert n_ready >= 36  # with 30% fault rates and 5 attempts almost every document succeeds


def test_permanent_failure_marks_document_failed(tmp_path, monkeypatch):
    monkeypatch.setattr(inproc_mod, "next_retry", _fast_retry)
    faults.configure({"handler.analyze": 100})  # fail the first 100 calls
    try:
        async def go():
            d, bus = _stack(tmp_path)
            stop = asyncio.Event()
            ws = await _run_workers(d, bus, 1, stop)
            doc = await d.store.create_document("x.txt")
            await d.queue.enqueue(Task(type=TASK_PARSE, payload=json.dumps(
                {"document_id": doc.id, "filename": "x.txt", "content": "a b c"}).encode()))
            for _ in range(200):
                if (await d.store.get_document(doc.id)).status == "failed":
                    break
                await asyncio.sleep(0.02)
            stop.set()
            await asyncio.gather(*ws)
            return (await d.store.get_document(doc.id)).status
        assert asyncio.run(go()) == "failed"
    finally:
        faults.configure(None)


def test_fault_spec_parsing():
    faults.configure("queue.enqueue:2,cache.get:0")
    try:
        n = 0
        for _ in range(5):
            try:
                faults.maybe_fail("queue.enqueue")
            except faults.InjectedFault:
                n += 1
        assert n == 2
        faults.maybe_fail("cache.get")
    finally:
        faults.configure(None)


def test_concurrent_pipeline_under_asyncio_debug(tmp_path, monkeypatch):
    """the ingest pipeline under asyncio debug mode with coroutine/resource warnings
    promoted to errors (a never-awaited coroutine or an un-closed resource fails the test)."""
    import warnings
    monkeypatch.setattr(inproc_mod, "next_retry", _fast_retry)

    async def go():
        d, bus = _stack(tmp_path)
        stop = asyncio.Event()
        ws = await _run_workers(d, bus, 2, stop)
        docs = []
        for i in range(12):
            doc = await d.store.create_document(f"g{i}.txt")
            docs.append(doc.id)
            await d.queue.enqueue(Task(type=TASK_PARSE, payload=json.dumps(
                {"document_id": doc.id, "filename": f"g{i}.txt", "content": "w " * 500}).encode()))
        for _ in range(400):
            st = [(await d.store.get_document(x)).status for x in docs]
            if all(v == "ready" for v in st):
                break
            await asyncio.sleep(0.02)
        stop.set()
        await asyncio.gather(*ws)
        return [(await d.store.get_document(x)).status for x in docs]

    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        statuses = asyncio.run(go(), debug=True)
    assert statuses == ["ready"] * 12


def test_search_results_resolved_in_one_query(tmp_path):
    """top_k hits -> chunks + their document's summary (or an empty one) + decoder tokens, in hit
    order, from ONE metadata query (store/sqlite_store.py _results)."""
    import numpy as np

    from docagents_amd.store.base import Chunk, Embedding, Summary

    async def go():
        meta = SqliteMeta(str(tmp_path / "m.sqlite3"))
        store = CompositeStore(meta, SqliteVectors(meta), min_similarity=-1.0)
        a = await store.create_document("a.txt")
        b = await store.create_document("b.txt")
        ca = await store.save_chunks(a.id, [Chunk(index=i, text=f"a{i}", token_count=1) for i in range(3)])
        cb = await store.save_chunks(b.id, [Chunk(index=0, text="b0", token_count=1)])
        await store.save_summary(a.id, Summary(a.id, "sum a", ["p1", "p2"]))
        await store.save_chunk_tokens([(ca[1].id, [7, 8, 9])])
        rng = np.random.default_rng(0)
        vecs = {c.id: rng.standard_normal(16).astype(np.float32) for c in ca + cb}
        vecs = {k: v / np.linalg.norm(v) for k, v in vecs.items()}
        await store.save_embeddings([Embedding(cid, v, "m") for cid, v in vecs.items()])
        calls = []
        orig = meta.q
        meta.q = lambda sql, args=(): (calls.append(sql), orig(sql, args))[1]
        res = await store.top_k([a.id, b.id], vecs[ca[1].id], 4)
        assert sum(1 for q in calls if "FROM chunks" in q or "FROM summaries" in q) == 1
        assert res[0].chunk.id == ca[1].id and res[0].score > 0.99
        assert {r.chunk.id for r in res} == {c.id for c in ca + cb}
        for r in res:
            assert r.tokens_loaded
            if r.chunk.document_id == a.id:
                assert (r.summary.summary, r.summary.key_points) == ("sum a", ["p1", "p2"])
            else:
                assert (r.summary.document_id, r.summary.summary, r.summary.key_points) == (b.id, "", [])
        assert np.frombuffer(res[0].tokens, dtype=np.int32).tolist() == [7, 8, 9]
        assert all(r.tokens is None for r in res[1:])
        assert await store.top_k([a.id], vecs[ca[0].id], 0) == []
        meta.close()
    asyncio.run(go())
