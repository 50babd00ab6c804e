"""Durable vector shards (index/wal.py; SURVEY §5.4, reference internal/store/postgres.go:176-201):
log framing + torn tails, checkpoint/rotation, and an engine process SIGKILLed mid-ingest that comes
back with every acknowledged document searchable at the same scores."""
import asyncio
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from docagents_amd.index.flat import FlatIndex
from docagents_amd.index.wal import ShardLog, scan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _unit(n, d, seed):
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(n, d, generator=g)
    return v / v.norm(dim=1, keepdim=True)


def _search_all(idx, q, doc_ids, k=4):
    s, rows = idx.search(q, k, -1.0, [doc_ids] * q.shape[0])
    return s.float().numpy(), idx.row_ids(rows.numpy().astype(np.int64))


def test_log_replay_checkpoint_and_torn_tail(tmp_path):
    d = 64
    idx = FlatIndex(d, "cpu")
    log = ShardLog(str(tmp_path), rank=3, fsync=False)
    assert log.recover(idx)["rows"] == 0
    vecs = {f"doc{i}": _unit(5, d, i) for i in range(6)}
    for i, (doc, v) in enumerate(vecs.items()):
        log.put(idx, doc, np.arange(5) + 10 * i, v)
    log.remove(idx, "doc2")
    log.put(idx, "doc4", np.arange(3) + 400, _unit(3, d, 99))  # re-index replaces the doc's rows
    log.checkpoint(idx)
    log.put(idx, "doc6", np.arange(5) + 60, _unit(5, d, 6))
    log.remove(idx, "doc0")
    log.close()
    # a crash mid-append: half a record at the end of the live log
    wal = os.path.join(str(tmp_path), f"shard3.wal.{log.gen}")
    with open(wal, "ab") as f:
        f.write(b"DAVL\x00\x10\x00\x00garbage")
    docs = [f"doc{i}" for i in range(7)]
    q = _unit(3, d, 1234)
    ref = _search_all(idx, q, docs)

    idx2 = FlatIndex(d, "cpu")
    log2 = ShardLog(str(tmp_path), rank=3, fsync=False)
    rec = log2.recover(idx2)
    assert rec["replayed"] == 2 and rec["torn_bytes"] > 0 and rec["snapshot_rows"] > 0
    got = _search_all(idx2, q, docs)
    np.testing.assert_array_equal(ref[1], got[1])
    np.testing.assert_allclose(ref[0], got[0], rtol=0, atol=1e-6)
    assert idx2.docs["doc2"].rows == 0 and idx2.docs["doc0"].rows == 0 and idx2.docs["doc4"].rows == 3
    # the torn tail was cut, so appends after recovery stay readable
    log2.put(idx2, "doc7", np.arange(2) + 70, _unit(2, d, 7))
    log2.close()
    recs, good, total = scan(wal)
    assert good == total and [r[1] for r in recs] == ["doc6", "doc0", "doc7"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start_engine(tmp_path, port):
    env = dict(os.environ, EMBED_ARCH="tiny-enc", LLM_ARCH="tiny-dec", ENGINE_CONTINUOUS="0",
               INDEX_DIR=str(tmp_path / "index"), INDEX_CHECKPOINT_S="0.5", ENGINE_LIVENESS_INTERVAL="0",
               DATA_DIR=str(tmp_path), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    lf = open(tmp_path / f"engine_{port}.log", "w")
    return subprocess.Popen([sys.executable, "-m", "docagents_amd.services", "engine", "--listen",
                             f"tcp://127.0.0.1:{port}"], env=env, stdout=lf, stderr=subprocess.STDOUT, cwd=ROOT)


async def _client(port):
    from docagents_amd.engine.rpc import EngineClient
    return await EngineClient(f"tcp://127.0.0.1:{port}").connect(retries=240, delay=0.25)


def _texts(i, n):
    return [f"Document: doc{i}.txt\n\nchunk {j} of document {i} about topic {i * 7 + j}" for j in range(n)]


def test_engine_sigkill_mid_ingest_recovers_every_acknowledged_doc(tmp_path):
    port = _port()
    proc = _start_engine(tmp_path, port)
    acked: dict[str, int] = {}
    try:
        async def ingest():
            cl = await _client(port)
            qv = (await cl.call("embed", texts=["topic 15 question", "document 3"], preprocess=True))["vecs"]

            async def one(i):
                r = await cl.call("embed_index", doc_id=f"doc{i}", keys=np.arange(4, dtype=np.int64) + 100 * i,
                                  texts=_texts(i, 4))
                acked[f"doc{i}"] = r["rows"]
            # first wave fully acknowledged (some of it checkpointed), second wave killed mid-flight
            await asyncio.gather(*[one(i) for i in range(12)])
            await asyncio.sleep(1.2)  # >= one checkpoint
            await asyncio.gather(*[one(i) for i in range(12, 16)])
            before = await cl.call("search", vecs=qv, filters=[sorted(acked)] * 2, k=6, min_sim=-1.0)
            tasks = [asyncio.ensure_future(one(i)) for i in range(16, 40)]
            await asyncio.sleep(0.05)
            proc.send_signal(signal.SIGKILL)
            await asyncio.gather(*tasks, return_exceptions=True)
            await cl.close()
            return qv, before, dict(acked)
        qv, before, acked_then = asyncio.run(ingest())
        proc.wait(timeout=30)
        assert len(acked_then) >= 16 and all(v == 4 for v in acked_then.values())

        proc = _start_engine(tmp_path, port)

        async def check():
            cl = await _client(port)
            have = await cl.call("index_docs")
            after = await cl.call("search", vecs=qv, filters=[sorted(before_docs)] * 2, k=6, min_sim=-1.0)
            await cl.close()
            return have, after
        before_docs = [f"doc{i}" for i in range(16)]
        have, after = asyncio.run(check())
        for d in acked_then:  # every acknowledged document is back, with all its rows
            assert have.get(d) == 4, (d, have.get(d))
        np.testing.assert_array_equal(before["keys"], after["keys"])
        np.testing.assert_allclose(before["scores"], after["scores"], rtol=0, atol=1e-6)
    finally:
        if proc.poll() is None:
            proc.send_signal(signal.SIGTERM)
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                proc.kill()


def test_startup_sweep_reenqueues_ready_docs_without_vectors(tmp_path):
    from docagents_amd.services.runner import startup_sweep
    from docagents_amd.store.base import STATUS_READY, Chunk
    from docagents_amd.store.sqlite_store import CompositeStore, SqliteMeta
    from docagents_amd.utils.log import discard

    class Vec:
        async def doc_rows(self):
            return {docs[0]: 2}

    class Q:
        def __init__(self):
            self.sent = []

        async def enqueue(self, task):
            self.sent.append(task)

    class D:
        pass

    store = CompositeStore(SqliteMeta(str(tmp_path / "m.sqlite3")), Vec())
    deps = D()
    deps.store, deps.queue, deps.log = store, Q(), discard()

    async def go():
        out = []
        for name in ("a.txt", "b.txt"):
            d = await store.create_document(name)
            await store.save_chunks(d.id, [Chunk(index=0, text="x"), Chunk(index=1, text="y")])
            await store.update_document_status(d.id, STATUS_READY)
            out.append(d.id)
        return out
    docs = asyncio.run(go())
    asyncio.run(startup_sweep(deps))
    import json
    sent = [json.loads(t.payload)["document_id"] for t in deps.queue.sent]
    assert sent == [docs[1]]


def test_startup_sweep_skips_in_flight_documents_and_analyze_is_idempotent(tmp_path):
    """A 'processing' document younger than SWEEP_STUCK_AFTER_S is in flight (a worker starting
    while uploads arrive must not duplicate its task); an older one is re-driven (flagged "redrive"); a re-driven
    analyze delivery of a ready document is a no-op."""
    import types

    from docagents_amd.services.analysis import handle_analyze
    from docagents_amd.services.runner import startup_sweep
    from docagents_amd.store.base import STATUS_READY, Chunk
    from docagents_amd.store.sqlite_store import CompositeStore, SqliteMeta
    from docagents_amd.utils.log import discard

    class Q:
        def __init__(self):
            self.sent = []

        async def enqueue(self, task):
            self.sent.append(task)

    store = CompositeStore(SqliteMeta(str(tmp_path / "m.sqlite3")), None)

    async def mk():
        d = await store.create_document("p.txt")
        await store.save_chunks(d.id, [Chunk(index=0, text="x")])
        return d.id
    doc = asyncio.run(mk())
    import json
    for grace, want in ((600.0, []), (-1.0, [doc])):
        deps = types.SimpleNamespace(store=store, queue=Q(), log=discard(),
                                     config=types.SimpleNamespace(sweep_stuck_after_s=grace))
        asyncio.run(startup_sweep(deps))
        assert [json.loads(t.payload)["document_id"] for t in deps.queue.sent] == want

    class Boom:
        async def summarize(self, text):
            raise AssertionError("a ready document must not be summarized again")
    asyncio.run(store.update_document_status(doc, STATUS_READY))
    deps = types.SimpleNamespace(store=store, llm=Boom(), config=types.SimpleNamespace(chunk_overlap=0))
    asyncio.run(handle_analyze(deps, {"document_id": doc, "redrive": True}))


def test_bad_mutation_is_rejected_before_it_is_logged_and_restart_works(tmp_path):
    """A wrong-dim index_add must fail the call without touching the document's rows or the log,
    and the engine must come back after a restart (round-2 advisor finding, index/wal.py:177)."""
    d = 32
    idx = FlatIndex(d, "cpu")
    log = ShardLog(str(tmp_path), fsync=False)
    log.recover(idx)
    log.put(idx, "doc", np.arange(4), _unit(4, d, 1))
    with pytest.raises(ValueError, match="dim"):
        log.upsert(idx, "doc", np.arange(2) + 100, _unit(2, d + 8, 2))
    with pytest.raises(ValueError, match="keys"):
        log.put(idx, "doc", np.arange(3), _unit(2, d, 3))
    assert idx.docs["doc"].rows == 4 and log.stats["appended"] == 1
    log.close()
    idx2 = FlatIndex(d, "cpu")
    rec = ShardLog(str(tmp_path), fsync=False).recover(idx2)
    assert rec["rows"] == 4 and rec["quarantined"] == 0 and idx2.docs["doc"].rows == 4


def test_unappliable_record_is_quarantined_not_fatal(tmp_path):
    """A record that fails to apply on replay (e.g. written by an older build without validation)
    is skipped and counted; recovery continues with the records after it."""
    from docagents_amd.index.wal import OP_PUT, _encode
    d = 16
    log = ShardLog(str(tmp_path), fsync=False)
    log.recover(FlatIndex(d, "cpu"))
    log._append(_encode(OP_PUT, "bad", np.arange(2), _unit(2, d * 2, 5)))  # wrong dim, bypassing validation
    log.put(FlatIndex(d, "cpu"), "good", np.arange(3), _unit(3, d, 6))
    log.close()
    idx = FlatIndex(d, "cpu")
    log2 = ShardLog(str(tmp_path), fsync=False)
    rec = log2.recover(idx)
    assert rec["quarantined"] == 1 and rec["replayed"] == 1 and idx.docs["good"].rows == 3
    assert log2.quarantine[0]["doc"] == "bad"


def test_index_add_is_a_per_chunk_upsert(tmp_path):
    """SaveEmbeddings parity (postgres.go:197, ON CONFLICT (chunk_id)): saving two chunk subsets of
    one document keeps both; re-saving a chunk replaces only that chunk's row."""
    from docagents_amd.engine.engine import Engine
    from docagents_amd.engine.server import EngineGroup
    eng = Engine("tiny-enc", "tiny-dec", "cpu", load_llm=False)
    for durable in (False, True):
        eng.index = FlatIndex(eng.dim, "cpu")
        sl = ShardLog(str(tmp_path / f"d{durable}"), fsync=False) if durable else None
        if sl:
            sl.recover(eng.index)
        g = EngineGroup(eng, shard_log=sl)
        v = _unit(5, eng.dim, 7).numpy()
        g.execute("index_add", {"doc_id": "doc", "keys": np.array([1, 2, 3]), "vecs": v[:3]})
        g.execute("index_add", {"doc_id": "doc", "keys": np.array([4, 5]), "vecs": v[3:]})
        assert eng.index.docs["doc"].rows == 5
        g.execute("index_add", {"doc_id": "doc", "keys": np.array([2]), "vecs": v[4:5]})  # chunk 2 re-embedded
        assert eng.index.docs["doc"].rows == 5
        q = torch.from_numpy(v[4:5])
        s, rows = eng.index.search(q, 5, -1.0, [["doc"]])
        keys = eng.index.row_ids(rows.numpy().astype(np.int64))[0]
        assert sorted(keys.tolist()) == [1, 2, 3, 4, 5]
        top2 = set(keys[:2].tolist())
        assert top2 == {2, 5}  # chunk 2 now carries chunk 5's vector: both score 1.0
        s_all, rows_all = eng.index.search(q, 10, -1.0, None)
        assert (rows_all >= 0).sum() == 5  # the replaced row is gone from dense scans too
        if sl:
            sl.close()
            idx2 = FlatIndex(eng.dim, "cpu")
            ShardLog(str(tmp_path / f"d{durable}"), fsync=False).recover(idx2)
            assert idx2.docs["doc"].rows == 5


def test_checkpoint_fsyncs_snapshot_and_directory_before_deleting_logs(tmp_path, monkeypatch):
    calls = []
    real_fsync, real_remove = os.fsync, os.remove
    monkeypatch.setattr(os, "fsync", lambda fd: (calls.append(("fsync", os.readlink(f"/proc/self/fd/{fd}"))),
                                                 real_fsync(fd))[1])
    monkeypatch.setattr(os, "remove", lambda p: (calls.append(("remove", p)), real_remove(p))[1])
    d = 16
    idx = FlatIndex(d, "cpu")
    log = ShardLog(str(tmp_path), fsync=True)
    log.recover(idx)
    log.put(idx, "doc", np.arange(2), _unit(2, d, 1))
    calls.clear()
    log.checkpoint(idx)
    first_remove = next(i for i, c in enumerate(calls) if c[0] == "remove")
    synced = [c[1] for c in calls[:first_remove] if c[0] == "fsync"]
    assert any(p.endswith(".snap.tmp") for p in synced), synced       # snapshot file contents
    assert synced.count(os.path.abspath(str(tmp_path))) >= 1, synced  # directory (rename + new log)
