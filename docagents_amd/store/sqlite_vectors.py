"""CPU vector backend: float32 blobs in the SQLite metadata DB, exact brute-force cosine in numpy.

This is BASELINE.json config 1 ("stub random-vector embed -> CPU brute-force cosine", the no-GPU
plumbing configuration) and the exactness oracle for the HBM indexes. Every process that opens
the same DB file sees the same vectors, so it works across the multi-process agent topology
without the engine server.
"""
from __future__ import annotations

import asyncio

import numpy as np


class SqliteVectors:
    def __init__(self, meta):
        self.meta = meta
        with meta.lock:
            meta.conn.execute("CREATE TABLE IF NOT EXISTS vectors (key INTEGER PRIMARY KEY, document_id TEXT, "
                              "vec BLOB)")
            meta.conn.execute("CREATE INDEX IF NOT EXISTS vectors_doc ON vectors(document_id)")

    async def add(self, doc_id: str, keys: np.ndarray, vecs: np.ndarray):
        rows = [(int(k), doc_id, np.asarray(v, dtype=np.float32).tobytes()) for k, v in zip(keys, vecs)]

        def f():
            with self.meta.lock:
                self.meta.conn.executemany("INSERT INTO vectors(key, document_id, vec) VALUES(?,?,?) ON CONFLICT(key) "
                                           "DO UPDATE SET vec=excluded.vec, document_id=excluded.document_id", rows)
        await asyncio.to_thread(f)

    async def search(self, vector: np.ndarray, doc_ids: list[str], k: int, min_sim: float):
        def f():
            if not doc_ids:
                return []
            qs = ",".join("?" * len(doc_ids))
            rows = self.meta.q(f"SELECT key, vec FROM vectors WHERE document_id IN ({qs})", tuple(doc_ids))
            if not rows:
                return []
            keys = np.asarray([r[0] for r in rows], dtype=np.int64)
            X = np.stack([np.frombuffer(r[1], dtype=np.float32) for r in rows])
            q = np.asarray(vector, dtype=np.float32)
            s = X @ q  # vectors are unit-norm: cosine similarity = dot product (1 - cosine distance)
            m = s >= min_sim
            keys, s = keys[m], s[m]
            order = np.lexsort((keys, -s))[:k]
            return [(int(keys[i]), float(s[i])) for i in order]
        return await asyncio.to_thread(f)

    async def remove_doc(self, doc_id: str):
        await asyncio.to_thread(self.meta.x, "DELETE FROM vectors WHERE document_id=?", (doc_id,))
