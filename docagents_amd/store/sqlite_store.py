"""Metadata in SQLite (WAL) + vectors in the HBM index: the Postgres/pgvector replacement.

Schema mirrors internal/store/postgres.go:63-87 (documents / chunks / summaries / embedding model),
plus an integer ``key`` per chunk (the vector id in the HBM index), a dense integer ``seq`` per
document, and the chunk's decoder token ids (tokenized once at analysis, reused for every Answer
prompt). Fixes carried over from SURVEY.md Appendix B: ``list_chunks`` orders by ``ord`` (#7),
``save_chunks`` replaces a document's chunks in one transaction so a parse retry is idempotent
(#17), migrations take an exclusive lock and non-holders WAIT instead of skipping (§5.2).

Vectors go to a ``VectorBackend`` (in-process HBM index, or the engine server over RPC).
"""
from __future__ import annotations

import asyncio
import datetime as dt
import json
import os
import sqlite3
import threading
import uuid

import numpy as np

from ..utils import faults
from ..utils import timeline
from .base import (STATUS_PROCESSING, Chunk, Document, DocumentNotFound, Embedding, SearchResult, Summary,
                   SummaryNotFound)

SCHEMA = [
    """CREATE TABLE IF NOT EXISTS documents (
        id TEXT PRIMARY KEY, seq INTEGER UNIQUE, filename TEXT, status TEXT,
        created_at TEXT DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')))""",
    """CREATE TABLE IF NOT EXISTS chunks (
        key INTEGER PRIMARY KEY AUTOINCREMENT, id TEXT UNIQUE, document_id TEXT REFERENCES documents(id)
        ON DELETE CASCADE, ord INTEGER, text TEXT, token_count INTEGER, dec_tokens BLOB)""",
    "CREATE INDEX IF NOT EXISTS chunks_doc ON chunks(document_id, ord)",
    """CREATE TABLE IF NOT EXISTS summaries (
        document_id TEXT PRIMARY KEY REFERENCES documents(id) ON DELETE CASCADE, summary TEXT, key_points TEXT)""",
    """CREATE TABLE IF NOT EXISTS embeddings (
        chunk_id TEXT PRIMARY KEY REFERENCES chunks(id) ON DELETE CASCADE, model TEXT, dim INTEGER)""",
]


class SqliteMeta:
    def __init__(self, path: str):
        self.path = path
        if path != ":memory:":
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self.conn = sqlite3.connect(path, check_same_thread=False, timeout=30.0, isolation_level=None)
        self.conn.execute("PRAGMA journal_mode=WAL")
        self.conn.execute("PRAGMA synchronous=NORMAL")
        self.conn.execute("PRAGMA foreign_keys=ON")
        self.lock = threading.RLock()
        # reads (q) run on a per-thread read-only connection: WAL lets readers run beside each other
        # and beside the writer, so the query path's chunk lookups (one per question, from the
        # executor threads) do not queue on the writer's lock under load (a 128-request burst
        # queued ~30 ms there). ":memory:" databases are per-connection: they keep the one connection
        self._tl = threading.local()
        self._readers: list = []
        self._migrate()

    def _reader(self):
        if self.path == ":memory:":
            return None
        c = getattr(self._tl, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, check_same_thread=False, timeout=30.0, isolation_level=None)
            c.execute("PRAGMA query_only=ON")
            self._tl.conn = c
            with self.lock:
                self._readers.append(c)
        return c

    def _migrate(self):
        with self.lock:
            # BEGIN EXCLUSIVE blocks concurrent migrators until the holder commits (no skip-and-race)
            self.conn.execute("BEGIN EXCLUSIVE")
            try:
                for s in SCHEMA:
                    self.conn.execute(s)
                self.conn.execute("COMMIT")
            except Exception:
                self.conn.execute("ROLLBACK")
                raise

    def q(self, sql, args=()):
        c = self._reader()
        if c is not None:
            return c.execute(sql, args).fetchall()
        with self.lock:
            return self.conn.execute(sql, args).fetchall()

    def x(self, sql, args=()):
        with self.lock:
            return self.conn.execute(sql, args)

    def close(self):
        with self.lock:
            for c in self._readers:
                c.close()
            self._readers.clear()
            self.conn.close()


def _parse_ts(s):
    if not s:
        return None
    try:
        return dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
    except ValueError:
        return None


class CompositeStore:
    """Store implementation: SQLite metadata + a vector backend (see vectors.py)."""

    def __init__(self, meta: SqliteMeta, vectors, min_similarity: float = 0.7, dec_tokenizer=None,
                 direct_embed: bool = False):
        self.meta, self.vectors = meta, vectors
        self.min_similarity = min_similarity
        self.dec_tokenizer = dec_tokenizer
        # the embedder and the vector shards are the same engine: EmbedBatch + SaveEmbeddings run as
        # one engine step that writes the rows into HBM directly (embed_and_save)
        self.direct_embed = direct_embed and hasattr(vectors, "embed_index")

    INLINE_LOOKUP_KEYS = 32  # _results: the question path's chunk lookup runs inline up to this many keys

    async def _run(self, fn, *a):
        return await asyncio.to_thread(fn, *a)

    # -------------------------------------------------------------------- documents
    async def create_document(self, filename: str) -> Document:
        def f():
            did = str(uuid.uuid4())
            with self.meta.lock:
                row = self.meta.conn.execute("SELECT COALESCE(MAX(seq), -1) + 1 FROM documents").fetchone()
                self.meta.conn.execute("INSERT INTO documents(id, seq, filename, status) VALUES(?,?,?,?)",
                                       (did, row[0], filename, STATUS_PROCESSING))
            return Document(did, filename, STATUS_PROCESSING, dt.datetime.now(dt.timezone.utc), row[0])
        return await self._run(f)

    async def get_document(self, doc_id: str) -> Document:
        rows = await self._run(self.meta.q, "SELECT id, filename, status, created_at, seq FROM documents WHERE id=?",
                               (doc_id,))
        if not rows:
            raise DocumentNotFound()
        r = rows[0]
        return Document(r[0], r[1], r[2], _parse_ts(r[3]), r[4])

    async def update_document_status(self, doc_id: str, status: str) -> None:
        cur = await self._run(self.meta.x, "UPDATE documents SET status=? WHERE id=?", (status, doc_id))
        if cur.rowcount == 0:
            raise DocumentNotFound()

    async def list_documents(self, status: str | None = None) -> list[Document]:
        sql = "SELECT id, filename, status, created_at, seq FROM documents"
        args = ()
        if status:
            sql += " WHERE status=?"
            args = (status,)
        rows = await self._run(self.meta.q, sql, args)
        return [Document(r[0], r[1], r[2], _parse_ts(r[3]), r[4]) for r in rows]

    # -------------------------------------------------------------------- chunks
    async def save_chunks(self, doc_id: str, chunks: list[Chunk]) -> list[Chunk]:
        faults.maybe_fail("store.save_chunks")

        def f():
            out = []
            with self.meta.lock:
                c = self.meta.conn
                c.execute("BEGIN IMMEDIATE")
                try:
                    c.execute("DELETE FROM chunks WHERE document_id=?", (doc_id,))
                    for ch in chunks:
                        cid = str(uuid.uuid4())
                        cur = c.execute("INSERT INTO chunks(id, document_id, ord, text, token_count) VALUES(?,?,?,?,?)",
                                        (cid, doc_id, ch.index, ch.text, ch.token_count))
                        out.append(Chunk(cid, doc_id, ch.index, ch.text, ch.token_count, cur.lastrowid))
                    c.execute("COMMIT")
                except Exception:
                    c.execute("ROLLBACK")
                    raise
            return out
        return await self._run(f)

    async def list_chunks(self, doc_id: str) -> list[Chunk]:
        rows = await self._run(self.meta.q, "SELECT id, ord, text, token_count, key FROM chunks WHERE document_id=? "
                                            "ORDER BY ord", (doc_id,))
        return [Chunk(r[0], doc_id, r[1], r[2], r[3], r[4]) for r in rows]

    async def chunks_by_keys(self, keys: list[int]) -> dict[int, tuple[Chunk, bytes | None]]:
        if not keys:
            return {}
        qs = ",".join("?" * len(keys))
        rows = await self._run(self.meta.q, f"SELECT key, id, document_id, ord, text, token_count, dec_tokens FROM chunks "
                                            f"WHERE key IN ({qs})", tuple(int(k) for k in keys))
        return {r[0]: (Chunk(r[1], r[2], r[3], r[4], r[5], r[0]), r[6]) for r in rows}

    async def save_chunk_tokens(self, pairs: list[tuple[str, list[int]]]):
        def f():
            with self.meta.lock:
                self.meta.conn.executemany("UPDATE chunks SET dec_tokens=? WHERE id=?",
                                           [(np.asarray(t, dtype=np.int32).tobytes(), cid) for cid, t in pairs])
        await self._run(f)

    # -------------------------------------------------------------------- summaries
    async def save_summary(self, doc_id: str, summary: Summary) -> None:
        await self._run(self.meta.x, "INSERT INTO summaries(document_id, summary, key_points) VALUES(?,?,?) "
                                     "ON CONFLICT(document_id) DO UPDATE SET summary=excluded.summary, "
                                     "key_points=excluded.key_points",
                        (doc_id, summary.summary, json.dumps(list(summary.key_points or []))))

    async def get_summary(self, doc_id: str) -> Summary:
        rows = await self._run(self.meta.q, "SELECT summary, key_points FROM summaries WHERE document_id=?", (doc_id,))
        if not rows:
            raise SummaryNotFound()
        return Summary(doc_id, rows[0][0], json.loads(rows[0][1] or "[]"))

    # -------------------------------------------------------------------- vectors
    async def save_embeddings(self, embs: list[Embedding]) -> None:
        if not embs:
            return
        ids = [e.chunk_id for e in embs]
        qs = ",".join("?" * len(ids))
        rows = await self._run(self.meta.q, f"SELECT id, key, document_id FROM chunks WHERE id IN ({qs})", tuple(ids))
        info = {r[0]: (r[1], r[2]) for r in rows}
        by_doc: dict[str, list] = {}
        for e in embs:
            if e.chunk_id not in info:
                raise LookupError(f"unknown chunk {e.chunk_id}")
            key, doc = info[e.chunk_id]
            by_doc.setdefault(doc, []).append((key, e.vector))
        for doc, items in by_doc.items():
            keys = np.asarray([k for k, _ in items], dtype=np.int64)
            vecs = np.stack([np.asarray(v, dtype=np.float32) for _, v in items])
            await self.vectors.add(doc, keys, vecs)

        def f():
            with self.meta.lock:
                self.meta.conn.executemany(
                    "INSERT INTO embeddings(chunk_id, model, dim) VALUES(?,?,?) ON CONFLICT(chunk_id) DO UPDATE SET "
                    "model=excluded.model, dim=excluded.dim",
                    [(e.chunk_id, e.model, int(np.asarray(e.vector).shape[-1])) for e in embs])
        await self._run(f)

    async def embed_and_save(self, doc_id: str, chunks: list[Chunk], texts: list[str], model: str) -> int:
        """EmbedBatch + SaveEmbeddings in one engine call (the vectors are written into the owner
        shard's HBM, durably logged there); records the embeddings metadata rows here."""
        rows, dim = await self.vectors.embed_index(doc_id, np.asarray([c.key for c in chunks], dtype=np.int64), texts)

        def f():
            with self.meta.lock:
                self.meta.conn.executemany(
                    "INSERT INTO embeddings(chunk_id, model, dim) VALUES(?,?,?) ON CONFLICT(chunk_id) DO UPDATE SET "
                    "model=excluded.model, dim=excluded.dim", [(c.id, model, dim) for c in chunks])
        await self._run(f)
        return rows

    async def top_k(self, doc_ids: list[str], vector, k: int, min_similarity: float | None = None) -> list[SearchResult]:
        thr = self.min_similarity if min_similarity is None else min_similarity
        hits = await self.vectors.search(np.asarray(vector, dtype=np.float32), list(doc_ids), k, thr)
        return await self._results(hits)

    @property
    def fused_query(self) -> bool:
        """Whether ``embed_top_k`` is available: the engine both embeds and holds the vectors."""
        return self.direct_embed and hasattr(self.vectors, "embed_search")

    async def embed_top_k(self, doc_ids: list[str], text: str, k: int, min_similarity: float | None = None):
        """Embed the (preprocessed) question AND search in ONE engine call (the question vector never
        leaves the engine between the two; cmd/query/main.go:87-105). Returns (vector, results)."""
        thr = self.min_similarity if min_similarity is None else min_similarity
        if timeline.enabled():
            timeline.mark("q_es_sent", t_text=text)
        vec, hits = await self.vectors.embed_search(text, list(doc_ids), k, thr)
        if timeline.enabled():
            timeline.mark("q_es_rx", t_text=text)
        res = await self._results(hits)
        if timeline.enabled():
            timeline.mark("q_results", t_text=text)
        return vec, res

    async def _results(self, hits) -> list[SearchResult]:
        """Chunks + their documents' summaries + decoder tokens of the hits in ONE query (one thread
        hop): under load every extra hop is a GIL / executor round trip on the question's path."""
        if not hits:
            return []
        keys = tuple(int(kk) for kk, _ in hits)
        qs = ",".join("?" * len(keys))
        sql = (f"SELECT c.key, c.id, c.document_id, c.ord, c.text, c.token_count, c.dec_tokens, s.document_id, "
               f"s.summary, s.key_points FROM chunks c LEFT JOIN summaries s ON s.document_id = c.document_id "
               f"WHERE c.key IN ({qs})")
        if len(keys) <= self.INLINE_LOOKUP_KEYS and self.meta.path != ":memory:":
            # a top-k's rows by primary key: ~0.1 ms in SQLite, cheaper inline (the event loop's own
            # read-only connection) than a thread-pool round trip, which under 128 in-flight queries
            # cost ~36 ms (profiles/r6/stack: chunk_rows)
            rows = self.meta.q(sql, keys)
        else:
            rows = await self._run(self.meta.q, sql, keys)
        found = {r[0]: r for r in rows}
        sums: dict[str, Summary] = {}
        out = []
        for key, score in hits:
            r = found.get(int(key))
            if r is None:
                continue
            doc = r[2]
            if doc not in sums:
                sums[doc] = Summary(doc, r[8], json.loads(r[9] or "[]")) if r[7] is not None else Summary(doc, "", [])
            out.append(SearchResult(Chunk(r[1], doc, r[3], r[4], r[5], r[0]), float(score), sums[doc],
                                    tokens=r[6], tokens_loaded=True))
        return out

    async def close(self):
        self.meta.close()
